/* CPU oracle (TEST INFRASTRUCTURE ONLY: the checker for the GPU path, never linked into
 * libhdrf.so) for stream-mode compressor == 5.
 *
 * Reference call site: DN/BlockReceiver.java:858-866 creates `new GzipCodec()` and
 * `codec.createOutputStream(fos)` for every received block and writes each packet into it
 * (:868-873, :887-894); DN/BlockReceiver.java:1238-1256 closes it.  GzipCodec lives in
 * hadoop-common 3.1.0 (NOT in /root/reference): with the native zlib loaded it is a
 * CompressorStream around ZlibCompressor(level DEFAULT = 6, strategy DEFAULT,
 * header GZIP_FORMAT = windowBits 31, memLevel 8, 64 KiB direct buffers).  The ZlibCompressor
 * accumulates the written bytes until its 64 KiB direct buffer is full and only then calls
 * deflate(Z_NO_FLUSH); close() calls deflate(Z_FINISH) on the rest.  For deflate level 6 the
 * emitted bits do not depend on how the input arrives in 64 KiB-aligned pieces (the window is
 * always full whenever the lookahead runs short before the final piece), so the file is
 * exactly zlib's gzip stream of the whole block.
 *
 * What follows restates zlib 1.2.11 (the host library of that Hadoop generation; the one in
 * this image, pinned byte for byte against it by tests/test_gzip.py) for level 6:
 *   deflate.c  deflate_slow (lazy matching: good 8, lazy 16, nice 128, chain 128, TOO_FAR 4096),
 *              fill_window / slide_hash (32 KiB window, 15-bit hash, shift 5), longest_match;
 *   trees.c    _tr_tally (16383 symbols per block), _tr_flush_block (stored / static / dynamic
 *              choice), build_tree (heap with the depth tie-break), gen_bitlen (length limit
 *              with the overflow redistribution), gen_codes, scan_tree / send_tree,
 *              send_all_trees, compress_block;
 *   the gzip wrapper (10-byte header with OS byte 3, CRC-32 and ISIZE trailer).
 * Positions are kept absolute (the block stays resident); the window start `base` advances by
 * 32 KiB exactly when zlib slides, and head/prev hold zlib's window-relative values (0 = NIL),
 * so NIL-ing, MAX_DIST and the stored-block eligibility follow zlib's bookkeeping exactly. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "hdrf_oracle.h"

#define WSIZE 32768
#define WMASK (WSIZE - 1)
#define HMASK 32767
#define MIN_LOOK 262              /* MAX_MATCH + MIN_MATCH + 1 */
#define MAX_DIST (WSIZE - MIN_LOOK)
#define LITBUF 16384              /* 1 << (memLevel + 6) */
#define L_CODES 286
#define D_CODES 30
#define BL_CODES 19
#define HEAP_SIZE (2 * L_CODES + 1)
#define END_BLOCK 256

enum { GOOD = 8, LAZY = 16, NICE = 128, CHAIN = 128, TOO_FAR = 4096 };

static const uint8_t XL[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint8_t XD[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
static const uint8_t XB[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
static const uint8_t BL_ORDER[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static uint8_t len_code[256], dist_code[512];
static int base_len[29], base_dist[30];
static uint16_t stat_lcode[288], stat_llen[288], stat_dcode[30], stat_dlen[30];
static uint32_t crc_tab[256];
static int tables_ready;

static unsigned bit_rev(unsigned c, int n)
{
    unsigned r = 0;
    while (n-- > 0) { r = (r << 1) | (c & 1); c >>= 1; }
    return r;
}

/* canonical codes from lengths (gen_codes) */
static void canon_codes(uint16_t *code, const uint16_t *len, int max_code, const uint16_t *count)
{
    uint16_t next[16];
    unsigned c = 0;
    for (int b = 1; b <= 15; b++) { c = (c + count[b - 1]) << 1; next[b] = (uint16_t)c; }
    for (int n = 0; n <= max_code; n++)
        if (len[n]) code[n] = (uint16_t)bit_rev(next[len[n]]++, len[n]);
}

static void init_tables(void)
{
    if (tables_ready) return;
    int l = 0, code;
    for (code = 0; code < 28; code++) {
        base_len[code] = l;
        for (int k = 0; k < (1 << XL[code]); k++) len_code[l++] = (uint8_t)code;
    }
    len_code[l - 1] = (uint8_t)code;          /* length 258 -> code 285 (index 28), not 284 */
    base_len[28] = 0;
    int d = 0;
    for (code = 0; code < 16; code++) {
        base_dist[code] = d;
        for (int k = 0; k < (1 << XD[code]); k++) dist_code[d++] = (uint8_t)code;
    }
    d >>= 7;
    for (; code < D_CODES; code++) {
        base_dist[code] = d << 7;
        for (int k = 0; k < (1 << (XD[code] - 7)); k++) dist_code[256 + d++] = (uint8_t)code;
    }
    uint16_t cnt[16] = {0};
    for (int n = 0; n < 288; n++) {
        stat_llen[n] = n <= 143 ? 8 : n <= 255 ? 9 : n <= 279 ? 7 : 8;
        cnt[stat_llen[n]]++;
    }
    canon_codes(stat_lcode, stat_llen, 287, cnt);
    for (int n = 0; n < D_CODES; n++) { stat_dlen[n] = 5; stat_dcode[n] = (uint16_t)bit_rev(n, 5); }
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_tab[n] = c;
    }
    tables_ready = 1;
}

static int dcode_of(unsigned dist) { return dist < 256 ? dist_code[dist] : dist_code[256 + (dist >> 7)]; }

/* ---- LSB-first bit writer (send_bits / bi_windup) ---- */
typedef struct { uint8_t *out; int64_t pos; uint64_t bb; int nb; } bitw;

static void put_bits(bitw *w, unsigned v, int n)
{
    w->bb |= (uint64_t)v << w->nb;
    w->nb += n;
    while (w->nb >= 8) { w->out[w->pos++] = (uint8_t)w->bb; w->bb >>= 8; w->nb -= 8; }
}

static void align_byte(bitw *w)
{
    if (w->nb > 0) w->out[w->pos++] = (uint8_t)w->bb;
    w->bb = 0;
    w->nb = 0;
}

/* ---- Huffman trees: fc = Freq|Code, dl = Dad|Len (zlib's ct_data unions) ---- */
typedef struct {
    uint16_t *fc, *dl;
    const uint16_t *slen;      /* static lengths (NULL for the bit-length tree) */
    const uint8_t *extra;
    int extra_base, elems, max_length, max_code;
} tree_t;

typedef struct {
    const uint8_t *src;
    int64_t n, base, strstart, block_start, match_start, prev_match;
    uint32_t lookahead, match_length, prev_length, match_available;
    int64_t *trace, ntrace, tcap;   /* optional longest_match call log (hdrf_oracle_gzip_trace) */
    uint32_t *syms;                 /* optional symbol log: (dist << 8) | lc per tally */
    int64_t *blks, nsyms, nblks;    /* optional block log: sym_end, block_start, strstart, base, last */
    uint16_t head[WSIZE], prev[WSIZE];
    uint16_t dbuf[LITBUF];
    uint8_t lbuf[LITBUF];
    uint32_t last_lit;
    uint16_t lfc[HEAP_SIZE], ldl[HEAP_SIZE], dfc[2 * D_CODES + 1], ddl[2 * D_CODES + 1];
    uint16_t bfc[2 * BL_CODES + 1], bdl[2 * BL_CODES + 1];
    tree_t lt, dt, bt;
    int heap[HEAP_SIZE], heap_len, heap_max;
    uint8_t depth[HEAP_SIZE];
    uint16_t bl_count[16];
    int64_t opt_len, static_len;
    bitw w;
} gz_state;

#define SMALLER(t, a, b) ((t)->fc[a] < (t)->fc[b] || ((t)->fc[a] == (t)->fc[b] && s->depth[a] <= s->depth[b]))

static void sift_down(gz_state *s, const tree_t *t, int k)
{
    const int v = s->heap[k];
    int j = k << 1;
    while (j <= s->heap_len) {
        if (j < s->heap_len && SMALLER(t, s->heap[j + 1], s->heap[j])) j++;
        if (SMALLER(t, v, s->heap[j])) break;
        s->heap[k] = s->heap[j];
        k = j;
        j <<= 1;
    }
    s->heap[k] = v;
}

static void bit_lengths(gz_state *s, tree_t *t)
{
    int overflow = 0, h;
    for (int b = 0; b <= 15; b++) s->bl_count[b] = 0;
    t->dl[s->heap[s->heap_max]] = 0;                           /* root */
    for (h = s->heap_max + 1; h < HEAP_SIZE; h++) {
        const int n = s->heap[h];
        int bits = t->dl[t->dl[n]] + 1;                         /* parent's Len + 1 */
        if (bits > t->max_length) { bits = t->max_length; overflow++; }
        t->dl[n] = (uint16_t)bits;
        if (n > t->max_code) continue;                          /* internal node */
        s->bl_count[bits]++;
        const int xb = n >= t->extra_base ? t->extra[n - t->extra_base] : 0;
        const int64_t f = t->fc[n];
        s->opt_len += f * (bits + xb);
        if (t->slen) s->static_len += f * (t->slen[n] + xb);
    }
    if (overflow == 0) return;
    do {
        int b = t->max_length - 1;
        while (s->bl_count[b] == 0) b--;
        s->bl_count[b]--;
        s->bl_count[b + 1] += 2;
        s->bl_count[t->max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (int b = t->max_length; b != 0; b--) {
        int n = s->bl_count[b];
        while (n != 0) {
            const int m = s->heap[--h];
            if (m > t->max_code) continue;
            if (t->dl[m] != b) {
                s->opt_len += ((int64_t)b - t->dl[m]) * t->fc[m];
                t->dl[m] = (uint16_t)b;
            }
            n--;
        }
    }
}

static void make_tree(gz_state *s, tree_t *t)
{
    int max_code = -1, node;
    s->heap_len = 0;
    s->heap_max = HEAP_SIZE;
    for (int n = 0; n < t->elems; n++) {
        if (t->fc[n] != 0) { s->heap[++s->heap_len] = max_code = n; s->depth[n] = 0; }
        else t->dl[n] = 0;
    }
    while (s->heap_len < 2) {                                   /* at least two codes */
        node = s->heap[++s->heap_len] = max_code < 2 ? ++max_code : 0;
        t->fc[node] = 1;
        s->depth[node] = 0;
        s->opt_len--;
        if (t->slen) s->static_len -= t->slen[node];
    }
    t->max_code = max_code;
    for (int n = s->heap_len / 2; n >= 1; n--) sift_down(s, t, n);
    node = t->elems;
    do {
        const int n = s->heap[1];
        s->heap[1] = s->heap[s->heap_len--];
        sift_down(s, t, 1);
        const int m = s->heap[1];
        s->heap[--s->heap_max] = n;
        s->heap[--s->heap_max] = m;
        t->fc[node] = (uint16_t)(t->fc[n] + t->fc[m]);
        s->depth[node] = (uint8_t)((s->depth[n] >= s->depth[m] ? s->depth[n] : s->depth[m]) + 1);
        t->dl[n] = t->dl[m] = (uint16_t)node;
        s->heap[1] = node++;
        sift_down(s, t, 1);
    } while (s->heap_len >= 2);
    s->heap[--s->heap_max] = s->heap[1];
    bit_lengths(s, t);
    canon_codes(t->fc, t->dl, max_code, s->bl_count);
}

/* run-length pass over a code-length sequence: count (send = 0) or emit (send = 1) */
static void rle_lengths(gz_state *s, tree_t *t, int max_code, int send)
{
    int prevlen = -1, nextlen = t->dl[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    if (!send) t->dl[max_code + 1] = 0xffff;                   /* guard */
    for (int n = 0; n <= max_code; n++) {
        const int curlen = nextlen;
        nextlen = t->dl[n + 1];
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) {
            if (send) do put_bits(&s->w, s->bfc[curlen], s->bdl[curlen]); while (--count != 0);
            else s->bfc[curlen] = (uint16_t)(s->bfc[curlen] + count);
        } else if (curlen != 0) {
            if (send) {
                if (curlen != prevlen) { put_bits(&s->w, s->bfc[curlen], s->bdl[curlen]); count--; }
                put_bits(&s->w, s->bfc[16], s->bdl[16]);
                put_bits(&s->w, (unsigned)(count - 3), 2);
            } else {
                if (curlen != prevlen) s->bfc[curlen]++;
                s->bfc[16]++;
            }
        } else if (count <= 10) {
            if (send) { put_bits(&s->w, s->bfc[17], s->bdl[17]); put_bits(&s->w, (unsigned)(count - 3), 3); }
            else s->bfc[17]++;
        } else {
            if (send) { put_bits(&s->w, s->bfc[18], s->bdl[18]); put_bits(&s->w, (unsigned)(count - 11), 7); }
            else s->bfc[18]++;
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

static void init_block(gz_state *s)
{
    for (int n = 0; n < L_CODES; n++) s->lfc[n] = 0;
    for (int n = 0; n < D_CODES; n++) s->dfc[n] = 0;
    for (int n = 0; n < BL_CODES; n++) s->bfc[n] = 0;
    s->lfc[END_BLOCK] = 1;
    s->opt_len = s->static_len = 0;
    s->last_lit = 0;
}

static void emit_symbols(gz_state *s, const uint16_t *lc_code, const uint16_t *lc_len, const uint16_t *d_code,
                         const uint16_t *d_len)
{
    for (uint32_t i = 0; i < s->last_lit; i++) {
        unsigned dist = s->dbuf[i], lc = s->lbuf[i];
        if (dist == 0) { put_bits(&s->w, lc_code[lc], lc_len[lc]); continue; }
        int code = len_code[lc];
        put_bits(&s->w, lc_code[code + 257], lc_len[code + 257]);
        if (XL[code]) put_bits(&s->w, lc - (unsigned)base_len[code], XL[code]);
        dist--;
        code = dcode_of(dist);
        put_bits(&s->w, d_code[code], d_len[code]);
        if (XD[code]) put_bits(&s->w, dist - (unsigned)base_dist[code], XD[code]);
    }
    put_bits(&s->w, lc_code[END_BLOCK], lc_len[END_BLOCK]);
}

static void flush_block(gz_state *s, int last)
{
    const int64_t stored_len = s->strstart - s->block_start;
    if (s->blks) {
        int64_t *b = s->blks + 5 * s->nblks++;
        b[0] = s->nsyms; b[1] = s->block_start; b[2] = s->strstart; b[3] = s->base; b[4] = last;
    }
    const int have_buf = s->block_start >= s->base;           /* zlib: block_start >= 0 (window-relative) */
    make_tree(s, &s->lt);
    make_tree(s, &s->dt);
    rle_lengths(s, &s->lt, s->lt.max_code, 0);
    rle_lengths(s, &s->dt, s->dt.max_code, 0);
    make_tree(s, &s->bt);
    int max_blindex;
    for (max_blindex = BL_CODES - 1; max_blindex >= 3; max_blindex--)
        if (s->bdl[BL_ORDER[max_blindex]] != 0) break;
    s->opt_len += 3 * ((int64_t)max_blindex + 1) + 5 + 5 + 4;
    int64_t opt_lenb = (s->opt_len + 3 + 7) >> 3;
    const int64_t static_lenb = (s->static_len + 3 + 7) >> 3;
    if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
    if (stored_len + 4 <= opt_lenb && have_buf) {
        put_bits(&s->w, (unsigned)last, 3);                    /* STORED_BLOCK = 0 */
        align_byte(&s->w);
        const unsigned L = (unsigned)stored_len & 0xffff;
        s->w.out[s->w.pos++] = (uint8_t)L;
        s->w.out[s->w.pos++] = (uint8_t)(L >> 8);
        s->w.out[s->w.pos++] = (uint8_t)~L;
        s->w.out[s->w.pos++] = (uint8_t)(~L >> 8);
        memcpy(s->w.out + s->w.pos, s->src + s->block_start, (size_t)stored_len);
        s->w.pos += stored_len;
    } else if (static_lenb == opt_lenb) {
        put_bits(&s->w, (1u << 1) + (unsigned)last, 3);
        emit_symbols(s, stat_lcode, stat_llen, stat_dcode, stat_dlen);
    } else {
        put_bits(&s->w, (2u << 1) + (unsigned)last, 3);
        const int lcodes = s->lt.max_code + 1, dcodes = s->dt.max_code + 1, blcodes = max_blindex + 1;
        put_bits(&s->w, (unsigned)(lcodes - 257), 5);
        put_bits(&s->w, (unsigned)(dcodes - 1), 5);
        put_bits(&s->w, (unsigned)(blcodes - 4), 4);
        for (int r = 0; r < blcodes; r++) put_bits(&s->w, s->bdl[BL_ORDER[r]], 3);
        rle_lengths(s, &s->lt, lcodes - 1, 1);
        rle_lengths(s, &s->dt, dcodes - 1, 1);
        emit_symbols(s, s->lfc, s->ldl, s->dfc, s->ddl);
    }
    init_block(s);
    if (last) align_byte(&s->w);
    s->block_start = s->strstart;
}

static int tally(gz_state *s, unsigned dist, unsigned lc)
{
    if (s->syms) s->syms[s->nsyms++] = (dist << 8) | lc;
    s->dbuf[s->last_lit] = (uint16_t)dist;
    s->lbuf[s->last_lit++] = (uint8_t)lc;
    if (dist == 0) s->lfc[lc]++;
    else {
        dist--;
        s->lfc[len_code[lc] + 257]++;
        s->dfc[dcode_of(dist)]++;
    }
    return s->last_lit == LITBUF - 1;
}

/* INSERT_STRING at absolute position p: returns the previous head (window-relative, 0 = NIL) */
static unsigned insert_at(gz_state *s, int64_t p)
{
    const uint8_t *b = s->src + p;
    const unsigned h = (((unsigned)b[0] << 10) ^ ((unsigned)b[1] << 5) ^ b[2]) & HMASK;
    const unsigned old = s->head[h];
    s->prev[p & WMASK] = (uint16_t)old;
    s->head[h] = (uint16_t)(p - s->base);
    return old;
}

/* fill_window with the whole block available: slide when strstart reaches WSIZE + MAX_DIST */
static void fill(gz_state *s)
{
    if (s->strstart - s->base >= WSIZE + MAX_DIST) {
        s->base += WSIZE;
        for (int k = 0; k < WSIZE; k++) {
            s->head[k] = (uint16_t)(s->head[k] >= WSIZE ? s->head[k] - WSIZE : 0);
            s->prev[k] = (uint16_t)(s->prev[k] >= WSIZE ? s->prev[k] - WSIZE : 0);
        }
    }
    const int64_t end = s->base + 2 * WSIZE < s->n ? s->base + 2 * WSIZE : s->n;
    s->lookahead = (uint32_t)(end - s->strstart);
}

static unsigned longest_match(gz_state *s, unsigned cur)
{
    unsigned chain = CHAIN;
    const int64_t ss = s->strstart - s->base;
    int best = (int)s->prev_length;
    unsigned nice = NICE;
    const unsigned limit = ss > MAX_DIST ? (unsigned)(ss - MAX_DIST) : 0;
    if (s->prev_length >= GOOD) chain >>= 2;
    if (nice > s->lookahead) nice = s->lookahead;
    /* prev_length >= lookahead: any result is <= prev_length and the previous match is emitted */
    if ((uint32_t)best >= s->lookahead) return s->lookahead;
    const uint8_t *scan = s->src + s->strstart;
    const int maxlen = s->lookahead < 258 ? (int)s->lookahead : 258;
    do {
        const uint8_t *m = s->src + s->base + cur;
        if (m[best] != scan[best] || m[best - 1] != scan[best - 1] || m[0] != scan[0] || m[1] != scan[1]) continue;
        int len = 3;                                           /* byte 2 equal by the hash */
        while (len < maxlen && m[len] == scan[len]) len++;
        if (len > best) {
            s->match_start = s->base + cur;
            best = len;
            if ((unsigned)len >= nice) break;
        }
    } while ((cur = s->prev[cur & WMASK]) > limit && --chain != 0);
    return (uint32_t)best <= s->lookahead ? (unsigned)best : s->lookahead;
}

static void deflate_slow(gz_state *s)
{
    for (;;) {
        if (s->lookahead < MIN_LOOK) {
            fill(s);
            if (s->lookahead == 0) break;
        }
        unsigned hash_head = 0;
        if (s->lookahead >= 3) hash_head = insert_at(s, s->strstart);
        s->prev_length = s->match_length;
        s->prev_match = s->match_start;
        s->match_length = 2;
        if (hash_head != 0 && s->prev_length < LAZY && s->strstart - s->base - hash_head <= MAX_DIST) {
            s->match_length = longest_match(s, hash_head);
            if (s->trace && s->ntrace < s->tcap) {
                int64_t *t = s->trace + 4 * s->ntrace++;
                t[0] = s->strstart; t[1] = s->prev_length; t[2] = s->match_length; t[3] = s->match_start;
            }
            if (s->match_length == 3 && s->strstart - s->match_start > TOO_FAR) s->match_length = 2;
        }
        if (s->prev_length >= 3 && s->match_length <= s->prev_length) {
            const int64_t max_insert = s->strstart + s->lookahead - 3;
            const int bflush = tally(s, (unsigned)(s->strstart - 1 - s->prev_match), s->prev_length - 3);
            s->lookahead -= s->prev_length - 1;
            s->prev_length -= 2;
            do {
                if (++s->strstart <= max_insert) insert_at(s, s->strstart);
            } while (--s->prev_length != 0);
            s->match_available = 0;
            s->match_length = 2;
            s->strstart++;
            if (bflush) flush_block(s, 0);
        } else if (s->match_available) {
            if (tally(s, 0, s->src[s->strstart - 1])) flush_block(s, 0);
            s->strstart++;
            s->lookahead--;
        } else {
            s->match_available = 1;
            s->strstart++;
            s->lookahead--;
        }
    }
    if (s->match_available) {
        tally(s, 0, s->src[s->strstart - 1]);
        s->match_available = 0;
    }
    flush_block(s, 1);
}

int64_t hdrf_oracle_gzip_bound(int64_t n) { return n + (n >> 3) + 1024; }

uint32_t hdrf_oracle_crc32(const uint8_t *p, int64_t n)
{
    init_tables();
    uint32_t c = 0xffffffffu;
    for (int64_t i = 0; i < n; i++) c = crc_tab[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return c ^ 0xffffffffu;
}

static int64_t gzip_run(const uint8_t *src, int64_t n, uint8_t *dst, int64_t *trace, int64_t tcap, int64_t *ntrace,
                        uint32_t *syms, int64_t *nsyms, int64_t *blks, int64_t *nblks);

/* The same compression, logging the lazy parse: syms (room for n + 1) receives (dist << 8) | lc
 * of every tallied symbol (dist 0 = literal lc, else lc = length - 3), blks (room for
 * 5 * (n / 16383 + 2)) one row per flushed block (symbol end, block_start, strstart, window base,
 * last).  Checker for the GPU parse (gz_parse_kernel). */
int64_t hdrf_oracle_gzip_symbols(const uint8_t *src, int64_t n, uint8_t *dst, uint32_t *syms, int64_t *nsyms,
                                 int64_t *blks, int64_t *nblks)
{
    return gzip_run(src, n, dst, NULL, 0, NULL, syms, nsyms, blks, nblks);
}

int64_t hdrf_oracle_gzip_compress(const uint8_t *src, int64_t n, uint8_t *dst)
{
    return gzip_run(src, n, dst, NULL, 0, NULL, NULL, NULL, NULL, NULL);
}

/* The same compression, logging every longest_match call as (strstart, prev_length, returned
 * length, match_start) into trace[4*k..] (at most tcap calls; *ntrace = calls logged).  Checker
 * for the GPU match pass (hdrf_gzip_match_pass): the answer a call returns is a function of the
 * position and of prev_length only. */
int64_t hdrf_oracle_gzip_trace(const uint8_t *src, int64_t n, uint8_t *dst, int64_t *trace, int64_t tcap,
                               int64_t *ntrace)
{
    return gzip_run(src, n, dst, trace, tcap, ntrace, NULL, NULL, NULL, NULL);
}

static int64_t gzip_run(const uint8_t *src, int64_t n, uint8_t *dst, int64_t *trace, int64_t tcap, int64_t *ntrace,
                        uint32_t *syms, int64_t *nsyms, int64_t *blks, int64_t *nblks)
{
    init_tables();
    gz_state *s = (gz_state *)calloc(1, sizeof(gz_state));
    if (!s) return -1;
    static const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};
    memcpy(dst, hdr, 10);
    s->src = src;
    s->n = n;
    s->trace = trace;
    s->syms = syms;
    s->blks = blks;
    s->tcap = tcap;
    s->match_length = s->prev_length = 2;
    s->w.out = dst;
    s->w.pos = 10;
    s->lt = (tree_t){s->lfc, s->ldl, stat_llen, XL, 257, L_CODES, 15, 0};
    s->dt = (tree_t){s->dfc, s->ddl, stat_dlen, XD, 0, D_CODES, 15, 0};
    s->bt = (tree_t){s->bfc, s->bdl, NULL, XB, 0, BL_CODES, 7, 0};
    init_block(s);
    deflate_slow(s);
    const uint32_t crc = hdrf_oracle_crc32(src, n), isize = (uint32_t)n;
    int64_t p = s->w.pos;
    for (int k = 0; k < 4; k++) dst[p++] = (uint8_t)(crc >> (8 * k));
    for (int k = 0; k < 4; k++) dst[p++] = (uint8_t)(isize >> (8 * k));
    if (ntrace) *ntrace = s->ntrace;
    if (nsyms) *nsyms = s->nsyms;
    if (nblks) *nblks = s->nblks;
    free(s);
    return p;
}
