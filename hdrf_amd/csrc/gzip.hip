// gzip.hip — stream-mode compressor 5 (Hadoop GzipCodec = zlib 1.2.11 level 6), stage 1 of the
// GPU deflate: the position-parallel match pass.
//
// Reference: DN/BlockReceiver.java:858-873,887-894 stream every received block through
// GzipCodec; the arithmetic is zlib's deflate_slow/longest_match (restated and pinned against
// zlib in oracle/hdrf_gzip.c, which is the checker of this file).  At level 6 every position
// p <= n-3 is inserted into the hash chains, the 15-bit hash is a pure function of the 3 bytes at
// p, and the lookahead mid-stream never drops under 262 B.  Hence longest_match(p) depends only on
// p and on whether prev_length >= good_match (chain 128, else 32; nice 128): the chain at p is
// "earlier positions with the same hash, nearest first", the head at distance <= MAX_DIST and
// every later candidate at distance < MAX_DIST, position 0 never (zlib's NIL).  The lazy parse
// (stage 2) then only reads the two answers computed here.
//
// gz_prev_kernel: prev[p] = 1 + nearest q < p with hash(q) == hash(p), q >= 1 (0: none within
//   MAX_DIST).  One workgroup per 4096-position tile: a 32768-entry "last position" table in LDS
//   (128 KiB) is seeded from the MAX_DIST positions before the tile (atomicMax, order-free), then
//   the tile runs in rounds of 256 positions (nearest equal hash earlier in the round, else the
//   table; the round's positions are then max-inserted).  Within a wave the nearest equal hash
//   comes from 16 ballots; the round's 4 waves read and insert in position order.
// gz_match_kernel: one lane per position walks prev[] and compares bytes; out128[p] / out32[p] =
//   (len << 16) | dist of the chain-128 / chain-32 answer (0 if no match of >= 3 bytes), bit 31
//   set when the head candidate sits at distance exactly MAX_DIST on a 32 KiB boundary — zlib's
//   window base after a slide is such a position and is NIL there, so stage 2 re-checks it.
#include "bytes.hpp"

namespace hdrf {

constexpr int kGzWsize = 32768;
constexpr int kGzMaxDist = kGzWsize - 262;       // MAX_DIST = WSIZE - MIN_LOOKAHEAD
constexpr int kGzTile = 4096;
constexpr int kGzHash = 1 << 15;

__device__ __forceinline__ uint32_t gz_hash(const uint8_t *s)
{
    return (((uint32_t)s[0] << 10) ^ ((uint32_t)s[1] << 5) ^ (uint32_t)s[2]) & (kGzHash - 1);
}

__global__ void __launch_bounds__(256) gz_prev_kernel(const uint8_t *__restrict__ src, int64_t n,
                                                      uint32_t *__restrict__ prev)
{
    extern __shared__ uint32_t last[];             // kGzHash entries: 1 + latest position (0 none)
    const int tid = threadIdx.x;
    const int64_t t0 = (int64_t)blockIdx.x * kGzTile;
    const int64_t nins = n - 2;                    // positions p <= n-3 are hashed/inserted
    for (int i = tid; i < kGzHash; i += 256) last[i] = 0;
    __syncthreads();
    int64_t w0 = t0 - kGzMaxDist;
    if (w0 < 1) w0 = 1;
    for (int64_t q = w0 + tid; q < t0 && q < nins; q += 256) atomicMax(&last[gz_hash(src + q)], (uint32_t)q + 1u);
    __syncthreads();
    const int lane = lane_id(), wave = tid >> 6;
    for (int r = 0; r < kGzTile; r += 256) {
        const int64_t p = t0 + r + tid;
        const bool valid = p < nins;
        const uint32_t h = valid ? gz_hash(src + p) : 0u;
        // lanes of this wave holding the same key (16 ballots); key bit 15 = not a candidate
        const uint32_t key = (valid && p >= 1) ? h : 0x8000u;
        uint64_t m = ~0ull;
        for (int bt = 0; bt < 16; bt++) {
            const uint64_t bal = __ballot((key >> bt) & 1u);
            m &= ((key >> bt) & 1u) ? bal : ~bal;
        }
        const uint64_t lower = lane ? m & ((1ull << lane) - 1ull) : 0ull;
        for (int w = 0; w < 4; w++) {                  // waves in position order: table, then insert
            if (wave == w && valid) {
                prev[p] = lower ? (uint32_t)(p - lane + (63 - __builtin_clzll(lower))) + 1u : last[h];
                if (p >= 1) atomicMax(&last[h], (uint32_t)p + 1u);
            }
            __syncthreads();
        }
    }
}

__global__ void __launch_bounds__(256) gz_match_kernel(const uint8_t *__restrict__ src, int64_t n,
                                                       const uint32_t *__restrict__ prev, uint32_t *__restrict__ out128,
                                                       uint32_t *__restrict__ out32)
{
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    uint32_t r128 = 0, r32 = 0;
    const uint32_t head = p < n - 2 ? prev[p] : 0u;
    if (head != 0 && p - (int64_t)(head - 1) <= kGzMaxDist) {
        const int64_t look = n - p;
        const int maxlen = look < 258 ? (int)look : 258;
        const int nice = look < 128 ? (int)look : 128;
        const uint8_t *scan = src + p;
        int best = 2, k = 0;
        int64_t bq = 0;
        uint32_t s32 = 0;
        bool snap = false;
        int64_t q = head - 1;
        uint32_t flag = (p - q == kGzMaxDist && (q & (kGzWsize - 1)) == 0) ? 0x80000000u : 0u;
        for (;;) {
            ++k;
            const uint8_t *m = src + q;
            int len = 0;
            while (len < maxlen && m[len] == scan[len]) len++;
            bool brk = false;
            if (len > best) {
                best = len;
                bq = q;
                brk = len >= nice;
            }
            if (k == 32) {
                s32 = best >= 3 ? ((uint32_t)best << 16) | (uint32_t)(p - bq) : 0u;
                snap = true;
            }
            if (brk || k == 128) break;
            const uint32_t nx = prev[q];
            if (nx == 0 || p - (int64_t)(nx - 1) >= kGzMaxDist) break;
            q = nx - 1;
        }
        r128 = best >= 3 ? ((uint32_t)best << 16) | (uint32_t)(p - bq) : 0u;
        r32 = snap ? s32 : r128;
        r128 |= flag;
        r32 |= flag;
    }
    out128[p] = r128;
    out32[p] = r32;
}

// ---- stage 2: zlib's lazy parse (deflate_slow) over the stage-1 answers, made segment-parallel.
// Everything a parse step reads besides its state is a function of the position: the window base
// (zlib slides at the first visited s > k*WSIZE + MAX_DIST, or at s == that threshold when fewer
// than 262 bytes remain — steps never jump 262 B), the "lookahead >= 3" test (n - s >= 3) and the
// stage-1 answers.  The state at the top of a step is (s, match_length, match_start,
// match_available).  So (a) one lane per 4096-position segment parses speculatively from a fresh
// state, recording the state and its symbol count at every position it visits; (b) one lane
// replays the true parse and, at the first position where its state equals the recorded one,
// jumps to that segment's exit (paths that meet stay together); (c) the segments' symbols
// (true-lane prefix + speculative rest) are concatenated, and the deflate blocks follow from
// the symbol count (a cut every 16,383 in-loop symbols) and the symbols' end positions.
constexpr int kGzSeg = 4096, kGzSegCap = kGzSeg + 2;

struct GzPs { uint32_t ml, ms, avail; };                 // match_length, match_start, match_available

__device__ __forceinline__ int64_t gz_base_at(int64_t s, int64_t n)
{
    int64_t k = 0;
    for (;;) {
        const int64_t T = (k + 1) * kGzWsize + kGzMaxDist;
        if (s > T || (s == T && n - s < 262)) k++;
        else break;
    }
    return k * kGzWsize;
}

__device__ __forceinline__ uint32_t gz_enc(const GzPs &q, int64_t s)
{
    const uint32_t d = q.ml >= 3 ? (uint32_t)(s - (int64_t)q.ms) & 0xffffu : 0u;
    return 0x80000000u | (q.avail << 30) | (q.ml << 16) | d;
}

// one step of deflate_slow at s (the top-of-loop fill already reflected in gz_base_at); emits
// at most one symbol via out(sym, end); returns the next s
template <class Out>
__device__ __forceinline__ int64_t gz_step(const uint8_t *src, int64_t n, const uint32_t *m128, const uint32_t *m32,
                                           int64_t s, GzPs &q, Out out)
{
    const uint32_t prev_length = q.ml, prev_match = q.ms;
    uint32_t ml = 2;
    if (n - s >= 3 && prev_length < 16) {
        const uint32_t v = (prev_length >= 8 ? m32 : m128)[s];
        const int64_t dist = v & 0xffff;
        const uint32_t len = (v >> 16) & 0x7fff;
        const bool nil = (v >> 31) && s - dist == gz_base_at(s, n);
        if (v && !nil && len > prev_length) {
            ml = len;
            q.ms = (uint32_t)(s - dist);
            if (len == 3 && dist > 4096) ml = 2;
        }
    }
    if (prev_length >= 3 && ml <= prev_length) {
        out(((uint32_t)(s - 1 - prev_match) << 8) | (prev_length - 3), (uint32_t)(s - 1 + prev_length));
        q.avail = 0;
        q.ml = 2;
        return s + prev_length - 1;
    }
    q.ml = ml;
    if (q.avail) out((uint32_t)src[s - 1], (uint32_t)s);
    q.avail = 1;
    return s + 1;
}

// (a) speculative lanes: st[s] / cn[s] = state and symbol count on arrival at s; ex[k] = exit
__global__ void __launch_bounds__(64) gz_spec_kernel(const uint8_t *__restrict__ src, int64_t n,
                                                     const uint32_t *__restrict__ m128, const uint32_t *__restrict__ m32,
                                                     uint32_t *__restrict__ st, uint32_t *__restrict__ cn,
                                                     uint32_t *__restrict__ ssym, uint32_t *__restrict__ send,
                                                     uint32_t *__restrict__ ex, int nseg)
{
    const int k = blockIdx.x * 64 + threadIdx.x;
    if (k >= nseg) return;
    const int64_t p0 = (int64_t)k * kGzSeg, e = p0 + kGzSeg < n ? p0 + kGzSeg : n;
    GzPs q{2, 0, 0};
    uint32_t c = 0;
    uint32_t *ys = ssym + (int64_t)k * kGzSegCap, *ye = send + (int64_t)k * kGzSegCap;
    int64_t s = p0;
    while (s < e) {
        st[s] = gz_enc(q, s);
        cn[s] = c;
        s = gz_step(src, n, m128, m32, s, q, [&](uint32_t y, uint32_t end) { ys[c] = y; ye[c] = end; c++; });
    }
    uint32_t *x = ex + 4 * (int64_t)k;
    x[0] = (uint32_t)s; x[1] = q.ml; x[2] = q.ms | (q.avail << 31); x[3] = c;
}

// (b) the true lane: fx* = its own symbols per segment, take[k] = {own count, first speculative
// symbol used}; tail = {after-loop literal?, symbol, end, in-loop symbol count}
__global__ void gz_fix_kernel(const uint8_t *__restrict__ src, int64_t n, const uint32_t *__restrict__ m128,
                              const uint32_t *__restrict__ m32, const uint32_t *__restrict__ st,
                              const uint32_t *__restrict__ cn, const uint32_t *__restrict__ ex,
                              uint32_t *__restrict__ fsym, uint32_t *__restrict__ fend, uint32_t *__restrict__ take,
                              uint32_t *__restrict__ tail, int nseg)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int k = 0; k < nseg; k++) { take[2 * k] = 0; take[2 * k + 1] = ex[4 * k + 3]; }
    GzPs q{2, 0, 0};
    int64_t s = 0;
    uint32_t total = 0;
    while (s < n) {
        const int k = (int)(s / kGzSeg);
        if (st[s] == gz_enc(q, s)) {                       // met the speculative path: jump to its exit
            take[2 * k + 1] = cn[s];
            const uint32_t *x = ex + 4 * (int64_t)k;
            total += x[3] - cn[s];
            s = x[0];
            q.ml = x[1]; q.ms = x[2] & 0x7fffffffu; q.avail = x[2] >> 31;
            continue;
        }
        uint32_t *fy = fsym + (int64_t)k * kGzSegCap, *fe = fend + (int64_t)k * kGzSegCap;
        s = gz_step(src, n, m128, m32, s, q, [&](uint32_t y, uint32_t end) {
            fy[take[2 * k]] = y; fe[take[2 * k]] = end; take[2 * k]++; total++;
        });
    }
    tail[0] = q.avail;
    tail[1] = n ? (uint32_t)src[n - 1] : 0u;
    tail[2] = (uint32_t)n;
    tail[3] = total;
}

// (c) segment offsets (one lane), then one workgroup per segment copies its symbols in order
__global__ void gz_segoff_kernel(const uint32_t *__restrict__ ex, const uint32_t *__restrict__ take, int nseg,
                                 uint32_t *__restrict__ off)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint32_t o = 0;
    for (int k = 0; k < nseg; k++) {
        off[k] = o;
        o += take[2 * k] + (ex[4 * k + 3] - take[2 * k + 1]);
    }
    off[nseg] = o;
}

__global__ void __launch_bounds__(256) gz_gather_kernel(const uint32_t *__restrict__ ssym, const uint32_t *__restrict__ send,
                                                        const uint32_t *__restrict__ fsym, const uint32_t *__restrict__ fend,
                                                        const uint32_t *__restrict__ ex, const uint32_t *__restrict__ take,
                                                        const uint32_t *__restrict__ off, uint32_t *__restrict__ syms,
                                                        uint32_t *__restrict__ symend)
{
    const int k = blockIdx.x;
    const int64_t base = (int64_t)k * kGzSegCap;
    const uint32_t nf = take[2 * k], from = take[2 * k + 1], to = ex[4 * k + 3], o = off[k];
    for (uint32_t i = threadIdx.x; i < nf; i += 256) { syms[o + i] = fsym[base + i]; symend[o + i] = fend[base + i]; }
    for (uint32_t i = from + threadIdx.x; i < to; i += 256) {
        syms[o + nf + i - from] = ssym[base + i];
        symend[o + nf + i - from] = send[base + i];
    }
}

// blocks: a cut after every 16,383rd in-loop symbol, then the last block (strstart = n)
__global__ void __launch_bounds__(256) gz_blocks_kernel(int64_t n, uint32_t *__restrict__ syms,
                                                        const uint32_t *__restrict__ symend, const uint32_t *__restrict__ tail,
                                                        int64_t *__restrict__ blks, int64_t *__restrict__ cnt)
{
    const uint32_t inloop = tail[3], total = inloop + tail[0];
    const int64_t ncut = inloop / 16383;
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b == 0) {
        if (tail[0]) syms[inloop] = tail[1];
        cnt[0] = total;
        cnt[1] = ncut + 1;
    }
    if (b > ncut) return;
    int64_t *r = blks + 5 * b;
    r[1] = b ? (int64_t)symend[b * 16383 - 1] : 0;
    if (b < ncut) {
        const int64_t j = (b + 1) * 16383 - 1;
        const uint32_t y = syms[j], end = symend[j];
        const int64_t cover = (y >> 8) ? (int64_t)(y & 0xff) + 3 : 1;
        r[0] = j + 1; r[2] = end; r[3] = gz_base_at(end - cover + 1, n); r[4] = 0;
    } else {
        r[0] = total; r[2] = n; r[3] = gz_base_at(n, n); r[4] = 1;
    }
}

size_t gzip_parse_scratch(int64_t n)
{
    const int64_t K = (n + kGzSeg - 1) / kGzSeg + 1;
    return (size_t)(8 * n + 16 * K * kGzSegCap + 16 * K + 8 * K + 16 + 4 * (n + 2) + 4 * (K + 1) + 1024);
}

hipError_t launch_gzip_parse(const uint8_t *src, int64_t n, const uint32_t *m128, const uint32_t *m32, uint32_t *syms,
                             int64_t *blks, int64_t *cnt, void *scratch, hipStream_t st)
{
    const int nseg = (int)((n + kGzSeg - 1) / kGzSeg);
    const int64_t K = nseg + 1;
    uint32_t *p = (uint32_t *)scratch;
    uint32_t *stw = p; p += n;
    uint32_t *cnw = p; p += n;
    uint32_t *ssym = p; p += K * kGzSegCap;
    uint32_t *send = p; p += K * kGzSegCap;
    uint32_t *fsym = p; p += K * kGzSegCap;
    uint32_t *fend = p; p += K * kGzSegCap;
    uint32_t *ex = p; p += 4 * K;
    uint32_t *take = p; p += 2 * K;
    uint32_t *tail = p; p += 4;
    uint32_t *symend = p; p += n + 2;
    uint32_t *off = p;
    if (n) if (hipError_t e = hipMemsetAsync(stw, 0, 4 * (size_t)n, st)) return e;
    if (nseg) {
        hipLaunchKernelGGL(gz_spec_kernel, dim3((nseg + 63) / 64), dim3(64), 0, st, src, n, m128, m32, stw, cnw, ssym,
                           send, ex, nseg);
    }
    hipLaunchKernelGGL(gz_fix_kernel, dim3(1), dim3(64), 0, st, src, n, m128, m32, stw, cnw, ex, fsym, fend, take, tail,
                       nseg);
    if (nseg) {
        hipLaunchKernelGGL(gz_segoff_kernel, dim3(1), dim3(64), 0, st, ex, take, nseg, off);
        hipLaunchKernelGGL(gz_gather_kernel, dim3(nseg), dim3(256), 0, st, ssym, send, fsym, fend, ex, take, off, syms,
                           symend);
    }
    const int64_t maxcut = n / 16383 + 1;
    hipLaunchKernelGGL(gz_blocks_kernel, dim3((unsigned)((maxcut + 255) / 256)), dim3(256), 0, st, n, syms, symend, tail,
                       blks, cnt);
    return hipGetLastError();
}

// ---- stage 3: one lane per deflate block builds zlib's trees (heap build_tree with the depth
// tie-break, gen_bitlen's overflow repair, scan_tree/bl_tree), makes the stored/static/dynamic
// choice of _tr_flush_block and writes the block's bits from bit 0 of its own scratch slot
// (stored blocks only record their length: their bits depend on the byte phase).
struct GzTab {
    uint8_t len_code[256], dist_code[512];
    int base_len[29], base_dist[30];
    uint16_t slcode[288], sllen[288], sdcode[30], sdlen[30];
    uint32_t crc64k[32];                               // CRC-32 shift by 64 KiB of zeros (GF(2) matrix)
};
struct GzBlk {
    uint16_t lfc[573], ldl[573], dfc[61], ddl[61], bfc[39], bdl[39];
    int heap[573];
    uint8_t depth[573];
    uint16_t bl_count[16];
    int heap_len, heap_max;
    int64_t opt_len, static_len;
};
struct GzTree { uint16_t *fc, *dl; const uint16_t *slen; const uint8_t *extra; int extra_base, elems, max_length, max_code; };
struct GzBits { uint8_t *out; int64_t pos; uint64_t bb; int nb; };

__constant__ uint8_t kGzXL[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint8_t kGzXD[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kGzXB[19] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 2, 3, 7};
__constant__ uint8_t kGzBlOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ void gz_put(GzBits &w, unsigned v, int n)
{
    w.bb |= (uint64_t)v << w.nb;
    w.nb += n;
    while (w.nb >= 8) { w.out[w.pos++] = (uint8_t)w.bb; w.bb >>= 8; w.nb -= 8; }
}

__device__ unsigned gz_rev(unsigned c, int n)
{
    unsigned r = 0;
    while (n-- > 0) { r = (r << 1) | (c & 1); c >>= 1; }
    return r;
}

__device__ bool gz_smaller(const GzTree &t, const GzBlk &s, int a, int b)
{
    return t.fc[a] < t.fc[b] || (t.fc[a] == t.fc[b] && s.depth[a] <= s.depth[b]);
}

__device__ void gz_sift(GzBlk &s, const GzTree &t, int k)
{
    const int v = s.heap[k];
    int j = k << 1;
    while (j <= s.heap_len) {
        if (j < s.heap_len && gz_smaller(t, s, s.heap[j + 1], s.heap[j])) j++;
        if (gz_smaller(t, s, v, s.heap[j])) break;
        s.heap[k] = s.heap[j];
        k = j;
        j <<= 1;
    }
    s.heap[k] = v;
}

__device__ void gz_bitlen(GzBlk &s, GzTree &t)
{
    int overflow = 0, h;
    for (int b = 0; b <= 15; b++) s.bl_count[b] = 0;
    t.dl[s.heap[s.heap_max]] = 0;
    for (h = s.heap_max + 1; h < 573; h++) {
        const int n = s.heap[h];
        int bits = t.dl[t.dl[n]] + 1;
        if (bits > t.max_length) { bits = t.max_length; overflow++; }
        t.dl[n] = (uint16_t)bits;
        if (n > t.max_code) continue;
        s.bl_count[bits]++;
        const int xb = n >= t.extra_base ? t.extra[n - t.extra_base] : 0;
        const int64_t f = t.fc[n];
        s.opt_len += f * (bits + xb);
        if (t.slen) s.static_len += f * (t.slen[n] + xb);
    }
    if (overflow == 0) return;
    do {
        int b = t.max_length - 1;
        while (s.bl_count[b] == 0) b--;
        s.bl_count[b]--;
        s.bl_count[b + 1] += 2;
        s.bl_count[t.max_length]--;
        overflow -= 2;
    } while (overflow > 0);
    for (int b = t.max_length; b != 0; b--) {
        int n = s.bl_count[b];
        while (n != 0) {
            const int m = s.heap[--h];
            if (m > t.max_code) continue;
            if (t.dl[m] != b) {
                s.opt_len += ((int64_t)b - t.dl[m]) * t.fc[m];
                t.dl[m] = (uint16_t)b;
            }
            n--;
        }
    }
}

__device__ void gz_tree(GzBlk &s, GzTree &t)
{
    int max_code = -1, node;
    s.heap_len = 0;
    s.heap_max = 573;
    for (int n = 0; n < t.elems; n++) {
        if (t.fc[n] != 0) { s.heap[++s.heap_len] = max_code = n; s.depth[n] = 0; }
        else t.dl[n] = 0;
    }
    while (s.heap_len < 2) {
        node = s.heap[++s.heap_len] = max_code < 2 ? ++max_code : 0;
        t.fc[node] = 1;
        s.depth[node] = 0;
        s.opt_len--;
        if (t.slen) s.static_len -= t.slen[node];
    }
    t.max_code = max_code;
    for (int n = s.heap_len / 2; n >= 1; n--) gz_sift(s, t, n);
    node = t.elems;
    do {
        const int n = s.heap[1];
        s.heap[1] = s.heap[s.heap_len--];
        gz_sift(s, t, 1);
        const int m = s.heap[1];
        s.heap[--s.heap_max] = n;
        s.heap[--s.heap_max] = m;
        t.fc[node] = (uint16_t)(t.fc[n] + t.fc[m]);
        s.depth[node] = (uint8_t)((s.depth[n] >= s.depth[m] ? s.depth[n] : s.depth[m]) + 1);
        t.dl[n] = t.dl[m] = (uint16_t)node;
        s.heap[1] = node++;
        gz_sift(s, t, 1);
    } while (s.heap_len >= 2);
    s.heap[--s.heap_max] = s.heap[1];
    gz_bitlen(s, t);
    uint16_t next[16];
    unsigned c = 0;
    for (int b = 1; b <= 15; b++) { c = (c + s.bl_count[b - 1]) << 1; next[b] = (uint16_t)c; }
    for (int n = 0; n <= max_code; n++)
        if (t.dl[n]) t.fc[n] = (uint16_t)gz_rev(next[t.dl[n]]++, t.dl[n]);
}

__device__ void gz_rle(GzBlk &s, GzTree &t, int max_code, GzBits *w)
{
    int prevlen = -1, nextlen = t.dl[0], count = 0, max_count = 7, min_count = 4;
    if (nextlen == 0) { max_count = 138; min_count = 3; }
    if (!w) t.dl[max_code + 1] = 0xffff;
    for (int n = 0; n <= max_code; n++) {
        const int curlen = nextlen;
        nextlen = t.dl[n + 1];
        if (++count < max_count && curlen == nextlen) continue;
        if (count < min_count) {
            if (w) do gz_put(*w, s.bfc[curlen], s.bdl[curlen]); while (--count != 0);
            else s.bfc[curlen] = (uint16_t)(s.bfc[curlen] + count);
        } else if (curlen != 0) {
            if (w) {
                if (curlen != prevlen) { gz_put(*w, s.bfc[curlen], s.bdl[curlen]); count--; }
                gz_put(*w, s.bfc[16], s.bdl[16]);
                gz_put(*w, (unsigned)(count - 3), 2);
            } else {
                if (curlen != prevlen) s.bfc[curlen]++;
                s.bfc[16]++;
            }
        } else if (count <= 10) {
            if (w) { gz_put(*w, s.bfc[17], s.bdl[17]); gz_put(*w, (unsigned)(count - 3), 3); }
            else s.bfc[17]++;
        } else {
            if (w) { gz_put(*w, s.bfc[18], s.bdl[18]); gz_put(*w, (unsigned)(count - 11), 7); }
            else s.bfc[18]++;
        }
        count = 0;
        prevlen = curlen;
        if (nextlen == 0) { max_count = 138; min_count = 3; }
        else if (curlen == nextlen) { max_count = 6; min_count = 3; }
        else { max_count = 7; min_count = 4; }
    }
}

__device__ __forceinline__ int gz_dcode(const GzTab &T, unsigned d) { return d < 256 ? T.dist_code[d] : T.dist_code[256 + (d >> 7)]; }

__device__ void gz_emit(GzBits &w, const GzTab &T, const uint32_t *sy, int64_t ns, const uint16_t *lcode,
                        const uint16_t *llen, const uint16_t *dcode, const uint16_t *dlen)
{
    for (int64_t i = 0; i < ns; i++) {
        unsigned dist = sy[i] >> 8, lc = sy[i] & 0xff;
        if (dist == 0) { gz_put(w, lcode[lc], llen[lc]); continue; }
        int code = T.len_code[lc];
        gz_put(w, lcode[code + 257], llen[code + 257]);
        if (kGzXL[code]) gz_put(w, lc - (unsigned)T.base_len[code], kGzXL[code]);
        dist--;
        code = gz_dcode(T, dist);
        gz_put(w, dcode[code], dlen[code]);
        if (kGzXD[code]) gz_put(w, dist - (unsigned)T.base_dist[code], kGzXD[code]);
    }
    gz_put(w, lcode[256], llen[256]);
}

__device__ __forceinline__ void gz_or_bits(uint8_t *base, int64_t bit, uint64_t v, int n)
{
    // v holds n <= 48 bits; OR them at bit offset `bit` (LSB-first) with 32-bit atomics
    while (n > 0) {
        const int64_t w = bit >> 5;
        const int sh = (int)(bit & 31);
        const int take = 32 - sh < n ? 32 - sh : n;
        const uint32_t part = (uint32_t)(v & ((1ull << take) - 1)) << sh;
        if (part) atomicOr((uint32_t *)base + w, part);
        v >>= take;
        n -= take;
        bit += take;
    }
}

// info[b] = {kind (0 stored, 1 static, 2 dynamic), bits (non-stored), stored_len}.  One workgroup
// per deflate block: lane 0 builds the trees, makes the choice and writes the block header and
// code-length codes; then the symbols are coded 256 at a time (bit lengths, a workgroup scan,
// ORed at their offsets).  The slot must be zero.
__global__ void __launch_bounds__(256) gz_block_kernel(const GzTab *__restrict__ tab, const uint32_t *__restrict__ syms,
                                                       const int64_t *__restrict__ blks, int nblk, GzBlk *__restrict__ st,
                                                       uint8_t *__restrict__ scratch, int64_t slot, int64_t *__restrict__ info)
{
    __shared__ int64_t s_bit;
    __shared__ int s_kind;
    __shared__ uint32_t s_wsum[4];
    const int b = blockIdx.x;
    const GzTab &T = *tab;
    GzBlk &s = st[b];
    const int64_t s0 = b ? blks[5 * (b - 1)] : 0, s1 = blks[5 * b];
    uint8_t *outp = scratch + (int64_t)b * slot;
    if (threadIdx.x == 0) {
        const int64_t *r = blks + 5 * b;
        const int last = (int)r[4];
        const int64_t stored_len = r[2] - r[1];
        const bool have_buf = r[1] >= r[3];
        for (int n = 0; n < 286; n++) s.lfc[n] = 0;
        for (int n = 0; n < 30; n++) s.dfc[n] = 0;
        for (int n = 0; n < 19; n++) s.bfc[n] = 0;
        s.lfc[256] = 1;
        s.opt_len = s.static_len = 0;
        for (int64_t i = s0; i < s1; i++) {
            const unsigned dist = syms[i] >> 8, lc = syms[i] & 0xff;
            if (dist == 0) s.lfc[lc]++;
            else { s.lfc[T.len_code[lc] + 257]++; s.dfc[gz_dcode(T, dist - 1)]++; }
        }
        GzTree lt{s.lfc, s.ldl, T.sllen, kGzXL, 257, 286, 15, 0};
        GzTree dt{s.dfc, s.ddl, T.sdlen, kGzXD, 0, 30, 15, 0};
        GzTree bt{s.bfc, s.bdl, nullptr, kGzXB, 0, 19, 7, 0};
        gz_tree(s, lt);
        gz_tree(s, dt);
        gz_rle(s, lt, lt.max_code, nullptr);
        gz_rle(s, dt, dt.max_code, nullptr);
        gz_tree(s, bt);
        int max_blindex;
        for (max_blindex = 18; max_blindex >= 3; max_blindex--)
            if (s.bdl[kGzBlOrder[max_blindex]] != 0) break;
        s.opt_len += 3 * ((int64_t)max_blindex + 1) + 14;
        int64_t opt_lenb = (s.opt_len + 10) >> 3;
        const int64_t static_lenb = (s.static_len + 10) >> 3;
        if (static_lenb <= opt_lenb) opt_lenb = static_lenb;
        int64_t *inf = info + 3 * b;
        inf[2] = stored_len;
        GzBits w{outp, 0, 0, 0};
        if (stored_len + 4 <= opt_lenb && have_buf) {
            s_kind = 0;
        } else if (static_lenb == opt_lenb) {
            gz_put(w, 2u + (unsigned)last, 3);
            s_kind = 1;
        } else {
            gz_put(w, 4u + (unsigned)last, 3);
            const int lcodes = lt.max_code + 1, dcodes = dt.max_code + 1, blcodes = max_blindex + 1;
            gz_put(w, (unsigned)(lcodes - 257), 5);
            gz_put(w, (unsigned)(dcodes - 1), 5);
            gz_put(w, (unsigned)(blcodes - 4), 4);
            for (int k = 0; k < blcodes; k++) gz_put(w, s.bdl[kGzBlOrder[k]], 3);
            gz_rle(s, lt, lcodes - 1, &w);
            gz_rle(s, dt, dcodes - 1, &w);
            s_kind = 2;
        }
        if (w.nb) w.out[w.pos] = (uint8_t)w.bb;
        s_bit = w.pos * 8 + w.nb;
        inf[0] = s_kind;
    }
    __syncthreads();
    const int kind = s_kind;
    if (kind == 0) return;
    __threadfence_block();
    const uint16_t *lcode = kind == 1 ? T.slcode : s.lfc, *llen = kind == 1 ? T.sllen : s.ldl;
    const uint16_t *dcode = kind == 1 ? T.sdcode : s.dfc, *dlen = kind == 1 ? T.sdlen : s.ddl;
    int64_t bit = s_bit;
    for (int64_t c0 = s0; c0 < s1; c0 += 256) {
        const int64_t i = c0 + threadIdx.x;
        uint64_t v = 0;
        int nb = 0;
        if (i < s1) {
            unsigned dist = syms[i] >> 8, lc = syms[i] & 0xff;
            if (dist == 0) { v = lcode[lc]; nb = llen[lc]; }
            else {
                int code = T.len_code[lc];
                v = lcode[code + 257]; nb = llen[code + 257];
                if (kGzXL[code]) { v |= (uint64_t)(lc - (unsigned)T.base_len[code]) << nb; nb += kGzXL[code]; }
                dist--;
                code = gz_dcode(T, dist);
                v |= (uint64_t)dcode[code] << nb; nb += dlen[code];
                if (kGzXD[code]) { v |= (uint64_t)(dist - (unsigned)T.base_dist[code]) << nb; nb += kGzXD[code]; }
            }
        }
        const uint32_t incl = wave_incl_scan((uint32_t)nb);
        if (lane_id() == 63) s_wsum[threadIdx.x >> 6] = incl;
        __syncthreads();
        uint32_t pre = 0, tot = 0;
        for (int k = 0; k < 4; k++) { if (k < (int)(threadIdx.x >> 6)) pre += s_wsum[k]; tot += s_wsum[k]; }
        if (nb) gz_or_bits(outp, bit + pre + incl - nb, v, nb);
        bit += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        gz_or_bits(outp, bit, lcode[256], llen[256]);
        info[3 * b + 1] = bit + llen[256];
    }
}

// ---- stage 4: bit offsets (one lane: the stored blocks' padding depends on the byte phase), then
// one workgroup per block ORs its bits into the file at its offset (32-bit atomics at the seams).
__global__ void gz_offsets_kernel(const int64_t *__restrict__ info, int nblk, int64_t *__restrict__ off)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int64_t bit = 80;                                              // the 10-byte gzip header
    for (int b = 0; b < nblk; b++) {
        off[b] = bit;
        const int64_t *inf = info + 3 * b;
        if (inf[0] == 0) bit = ((bit + 3 + 7) & ~7ll) + 32 + 8 * inf[2];
        else bit += inf[1];
    }
    off[nblk] = (bit + 7) & ~7ll;                                  // last block: align_byte
}

__device__ __forceinline__ void gz_or_byte(uint8_t *out, int64_t byte, uint32_t v)
{
    if (!v) return;
    uint32_t *w = (uint32_t *)(out + (byte & ~3ll));
    atomicOr(w, v << (8 * (byte & 3)));
}

__global__ void __launch_bounds__(256) gz_place_kernel(const uint8_t *__restrict__ src, const int64_t *__restrict__ blks,
                                                       const int64_t *__restrict__ info, const int64_t *__restrict__ off,
                                                       const uint8_t *__restrict__ scratch, int64_t slot,
                                                       uint8_t *__restrict__ out)
{
    const int b = blockIdx.x;
    const int64_t *inf = info + 3 * b;
    const int64_t bit0 = off[b];
    if (inf[0] == 0) {
        const int last = (int)blks[5 * b + 4];
        const int64_t start = blks[5 * b + 1], len = inf[2];
        if (threadIdx.x == 0) {
            gz_or_byte(out, bit0 >> 3, (uint32_t)last << (bit0 & 7));   // 3 header bits (type 0)
            const int64_t pos = (bit0 + 3 + 7) >> 3;
            const unsigned L = (unsigned)len & 0xffff;
            gz_or_byte(out, pos, L & 0xff);
            gz_or_byte(out, pos + 1, L >> 8);
            gz_or_byte(out, pos + 2, (~L) & 0xff);
            gz_or_byte(out, pos + 3, (~L >> 8) & 0xff);
        }
        const int64_t pos = ((bit0 + 3 + 7) >> 3) + 4;
        for (int64_t i = threadIdx.x; i < len; i += 256) gz_or_byte(out, pos + i, src[start + i]);
        return;
    }
    const int64_t nbits = inf[1];
    const int64_t nbytes = (nbits + 7) >> 3;
    const int sh = (int)(bit0 & 7);
    const int64_t byte0 = bit0 >> 3;
    const uint8_t *in = scratch + (int64_t)b * slot;
    for (int64_t i = threadIdx.x; i < nbytes; i += 256) {
        uint32_t v = in[i];
        if (8 * (i + 1) > nbits) v &= (1u << (nbits - 8 * i)) - 1u;  // bits past the block end
        v <<= sh;
        gz_or_byte(out, byte0 + i, v & 0xff);
        gz_or_byte(out, byte0 + i + 1, v >> 8);
    }
}

// CRC-32 (gzip trailer): per-64 KiB piece in parallel, then combined in order with zlib's
// crc32_combine (GF(2) matrix powers of the zero-byte operator) by one lane.
__device__ uint32_t gz_crc_table(int i)
{
    uint32_t c = (uint32_t)i;
    for (int k = 0; k < 8; k++) c = c & 1 ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    return c;
}

__global__ void __launch_bounds__(256) gz_crc_piece_kernel(const uint8_t *__restrict__ src, int64_t n,
                                                           uint32_t *__restrict__ pcrc)
{
    __shared__ uint32_t tab[256];
    tab[threadIdx.x] = gz_crc_table(threadIdx.x);
    __syncthreads();
    const int64_t pc = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t a = pc << 16, e = a + 65536 < n ? a + 65536 : n;
    if (a >= n) return;
    uint32_t c = 0xffffffffu;
    for (int64_t i = a; i < e; i++) c = tab[(c ^ src[i]) & 0xff] ^ (c >> 8);
    pcrc[pc] = c ^ 0xffffffffu;
}

__device__ uint32_t gz_mtimes(const uint32_t *m, uint32_t v)
{
    uint32_t s = 0;
    for (int i = 0; v; i++, v >>= 1) if (v & 1) s ^= m[i];
    return s;
}

__device__ void gz_msquare(uint32_t *sq, const uint32_t *m)
{
    for (int i = 0; i < 32; i++) sq[i] = gz_mtimes(m, m[i]);
}

__device__ uint32_t gz_crc_combine(uint32_t c1, uint32_t c2, int64_t len2)
{
    uint32_t even[32], odd[32];
    if (len2 <= 0) return c1;
    odd[0] = 0xedb88320u;
    uint32_t row = 1;
    for (int i = 1; i < 32; i++) { odd[i] = row; row <<= 1; }
    gz_msquare(even, odd);
    gz_msquare(odd, even);
    do {
        gz_msquare(even, odd);
        if (len2 & 1) c1 = gz_mtimes(even, c1);
        len2 >>= 1;
        if (len2 == 0) break;
        gz_msquare(odd, even);
        if (len2 & 1) c1 = gz_mtimes(odd, c1);
        len2 >>= 1;
    } while (len2 != 0);
    return c1 ^ c2;
}

__global__ void gz_trailer_kernel(const GzTab *__restrict__ tab, const uint32_t *__restrict__ pcrc, int64_t n,
                                  const int64_t *__restrict__ off, int nblk, uint8_t *__restrict__ out,
                                  int64_t *__restrict__ flen)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    __shared__ uint32_t M[32];
    for (int i = 0; i < 32; i++) M[i] = tab->crc64k[i];
    uint32_t c = 0;
    for (int64_t a = 0, k = 0; a < n; a += 65536, k++) {
        const int64_t l = n - a < 65536 ? n - a : 65536;
        c = l == 65536 ? gz_mtimes(M, c) ^ pcrc[k] : gz_crc_combine(c, pcrc[k], l);
    }
    const int64_t p = off[nblk] >> 3;
    const uint8_t hdr[10] = {0x1f, 0x8b, 8, 0, 0, 0, 0, 0, 0, 3};
    for (int k = 0; k < 10; k++) gz_or_byte(out, k, hdr[k]);
    for (int k = 0; k < 4; k++) gz_or_byte(out, p + k, (c >> (8 * k)) & 0xff);
    for (int k = 0; k < 4; k++) gz_or_byte(out, p + 4 + k, ((uint32_t)n >> (8 * k)) & 0xff);
    *flen = p + 8;
}

size_t gzip_block_state_bytes() { return sizeof(GzBlk); }
size_t gzip_tab_bytes() { return sizeof(GzTab); }

void gzip_host_tab(void *dst)
{
    GzTab &T = *(GzTab *)dst;
    static const uint8_t XL[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
    static const uint8_t XD[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
    int l = 0, code;
    for (code = 0; code < 28; code++) {
        T.base_len[code] = l;
        for (int k = 0; k < (1 << XL[code]); k++) T.len_code[l++] = (uint8_t)code;
    }
    T.len_code[l - 1] = (uint8_t)code;
    T.base_len[28] = 0;
    int d = 0;
    for (code = 0; code < 16; code++) {
        T.base_dist[code] = d;
        for (int k = 0; k < (1 << XD[code]); k++) T.dist_code[d++] = (uint8_t)code;
    }
    d >>= 7;
    for (; code < 30; code++) {
        T.base_dist[code] = d << 7;
        for (int k = 0; k < (1 << (XD[code] - 7)); k++) T.dist_code[256 + d++] = (uint8_t)code;
    }
    uint16_t cnt[16] = {0}, next[16];
    for (int n = 0; n < 288; n++) {
        T.sllen[n] = n <= 143 ? 8 : n <= 255 ? 9 : n <= 279 ? 7 : 8;
        cnt[T.sllen[n]]++;
    }
    auto rev = [](unsigned c, int n) { unsigned r = 0; while (n-- > 0) { r = (r << 1) | (c & 1); c >>= 1; } return r; };
    unsigned c = 0;
    for (int b = 1; b <= 15; b++) { c = (c + cnt[b - 1]) << 1; next[b] = (uint16_t)c; }
    for (int n = 0; n < 288; n++) T.slcode[n] = (uint16_t)rev(next[T.sllen[n]]++, T.sllen[n]);
    for (int n = 0; n < 30; n++) { T.sdlen[n] = 5; T.sdcode[n] = (uint16_t)rev((unsigned)n, 5); }
    // zlib crc32_combine's operator for 65,536 zero bytes: odd = one zero bit, squared 3 times
    // gives one zero byte, then 16 more squarings give 2^16 bytes; column i = image of bit i
    auto times = [](const uint32_t *m, uint32_t v) { uint32_t r = 0; for (int i = 0; v; i++, v >>= 1) if (v & 1) r ^= m[i]; return r; };
    uint32_t op[32], sq[32];
    op[0] = 0xedb88320u;
    for (int i = 1; i < 32; i++) op[i] = 1u << (i - 1);
    for (int r = 0; r < 3 + 16; r++) {
        for (int i = 0; i < 32; i++) sq[i] = times(op, op[i]);
        for (int i = 0; i < 32; i++) op[i] = sq[i];
    }
    for (int i = 0; i < 32; i++) T.crc64k[i] = op[i];
}

hipError_t launch_gzip_encode(const uint8_t *src, int64_t n, const void *tab, const uint32_t *syms, const int64_t *blks,
                              int nblk, void *state, uint8_t *scratch, int64_t slot, int64_t *info, int64_t *off,
                              uint32_t *pcrc, uint8_t *out, int64_t *flen, hipStream_t st)
{
    if (hipError_t e = hipMemsetAsync(scratch, 0, (size_t)slot * (size_t)nblk, st)) return e;
    hipLaunchKernelGGL(gz_block_kernel, dim3(nblk), dim3(256), 0, st, (const GzTab *)tab, syms, blks, nblk,
                       (GzBlk *)state, scratch, slot, info);
    hipLaunchKernelGGL(gz_offsets_kernel, dim3(1), dim3(64), 0, st, info, nblk, off);
    hipLaunchKernelGGL(gz_place_kernel, dim3(nblk), dim3(256), 0, st, src, blks, info, off, scratch, slot, out);
    const int64_t pieces = (n + 65535) >> 16;
    if (pieces) hipLaunchKernelGGL(gz_crc_piece_kernel, dim3((unsigned)((pieces + 255) / 256)), dim3(256), 0, st, src, n, pcrc);
    hipLaunchKernelGGL(gz_trailer_kernel, dim3(1), dim3(64), 0, st, (const GzTab *)tab, pcrc, n, off, nblk, out, flen);
    return hipGetLastError();
}

size_t gzip_match_lds() { return sizeof(uint32_t) * kGzHash; }

hipError_t launch_gzip_match(const uint8_t *src, int64_t n, uint32_t *prev, uint32_t *out128, uint32_t *out32,
                             hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    static const hipError_t attr = hipFuncSetAttribute((const void *)gz_prev_kernel,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)gzip_match_lds());
    if (attr != hipSuccess) return attr;
    const unsigned tiles = (unsigned)((n + kGzTile - 1) / kGzTile);
    hipLaunchKernelGGL(gz_prev_kernel, dim3(tiles), dim3(256), gzip_match_lds(), st, src, n, prev);
    const unsigned g = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(gz_match_kernel, dim3(g), dim3(256), 0, st, src, n, prev, out128, out32);
    return hipGetLastError();
}

}  // namespace hdrf
