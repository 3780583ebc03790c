/*
 * hdrf_oracle.c — CPU restatement of HDRF's per-block reduction path.
 *
 * TEST INFRASTRUCTURE ONLY (see hdrf_oracle.h for the pinning status).
 * Every function cites the reference lines it restates.  `DN/` abbreviates
 * /root/reference/hadoop-hdfs/src/main/java/org/apache/hadoop/hdfs/server/datanode/.
 *
 * Redis (key/value server reached through Jedis 2.9.0, DN/DataDeduplicator.java:119)
 * is restated as in-memory maps with GET/SET semantics; container files under
 * DataNode.chunkDir are restated as in-memory byte vectors.
 */
#include "hdrf_oracle.h"
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* a1: DataDeduplicator.chunking — DN/DataDeduplicator.java:264-307 (literal transliteration). */
int64_t hdrf_oracle_chunk(const uint8_t *data, int64_t size, uint32_t *out, int64_t out_cap)
{
    const int w = 700;                                   /* :266 */
    const int mLength = 1000000;                         /* :272 */
    int8_t mValue = size > 0 ? (int8_t)data[0] : 0;     /* :268  data.get(0) (a fresh direct buffer reads 0) */
    int64_t mPos = w;                                    /* :269 */
    int64_t count = -1;                                  /* :270 */
    int64_t cLength = 0;                                 /* :271 */
    /* offsetarray has capacity/w + 1 slots (:267); we keep every detected boundary. */
    int64_t ocap = size / w + 2;
    uint32_t *offsetarray = (uint32_t *)malloc((size_t)ocap * sizeof(uint32_t));
    if (!offsetarray) return -2;
    for (int64_t i = 0; i < size; i++) {                 /* :274 */
        cLength++;                                       /* :275 */
        int8_t b = (int8_t)data[i];
        if (b >= mValue) {                               /* :276  signed Java byte compare */
            if (i > mPos) {                              /* :277 */
                count++;
                offsetarray[count] = (uint32_t)(i + 1);  /* :279 */
                mPos = i + w + 1;                        /* :280 */
                mValue = 0;                              /* :281 */
                cLength = 0;                             /* :282 */
                continue;                                /* :283 */
            } else {
                mValue = b;                              /* :285 */
            }
        }
        if (cLength > mLength) {                         /* :288-294 forced cut */
            count++;
            offsetarray[count] = (uint32_t)(i + 1);
            mPos = i + w + 1;
            mValue = 0;
            cLength = 0;
        }
    }
    /* :300-304 — the last detected boundary is dropped, then `size` is appended. */
    int64_t n = (count > 0 ? count : 0) + 1;
    if (n > out_cap) { free(offsetarray); return -1; }
    for (int64_t i = 0; i < count; i++) out[i] = offsetarray[i];
    out[n - 1] = (uint32_t)size;
    free(offsetarray);
    return n;
}

/* ------------------------------------------------------------------------------------------ */
/* a3: FIPS 180-4 SHA-1 and SHA-224 (utilities.sha1hash / sha224hash, DN/utilities.java:98-137;
 * the native path is nayuki's sha1_compress_block / sha256_compress_block + standard padding). */
static inline uint32_t rol32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static inline uint32_t ror32(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }
static inline uint32_t be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static void sha1_compress(uint32_t st[5], const uint8_t blk[64])
{
    uint32_t w[80];
    for (int i = 0; i < 16; i++) w[i] = be32(blk + 4 * i);
    for (int i = 16; i < 80; i++) w[i] = rol32(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
    for (int i = 0; i < 80; i++) {
        uint32_t f, k;
        if (i < 20)      { f = (b & c) | (~b & d);           k = 0x5A827999u; }
        else if (i < 40) { f = b ^ c ^ d;                    k = 0x6ED9EBA1u; }
        else if (i < 60) { f = (b & c) | (b & d) | (c & d);  k = 0x8F1BBCDCu; }
        else             { f = b ^ c ^ d;                    k = 0xCA62C1D6u; }
        uint32_t t = rol32(a, 5) + f + e + k + w[i];
        e = d; d = c; c = rol32(b, 30); b = a; a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static void sha256_compress(uint32_t st[8], const uint8_t blk[64])
{
    uint32_t w[64];
    for (int i = 0; i < 16; i++) w[i] = be32(blk + 4 * i);
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ror32(w[i - 15], 7) ^ ror32(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ror32(w[i - 2], 17) ^ ror32(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
    for (int i = 0; i < 64; i++) {
        uint32_t S1 = ror32(e, 6) ^ ror32(e, 11) ^ ror32(e, 25);
        uint32_t ch = (e & f) ^ (~e & g);
        uint32_t t1 = h + S1 + ch + K256[i] + w[i];
        uint32_t S0 = ror32(a, 2) ^ ror32(a, 13) ^ ror32(a, 22);
        uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
        uint32_t t2 = S0 + mj;
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

/* Merkle–Damgård padding shared by both hashes: 0x80, zeros, 64-bit big-endian bit length. */
static void md_hash(const uint8_t *msg, uint64_t len, uint32_t *st,
                    void (*compress)(uint32_t *, const uint8_t *))
{
    uint64_t full = len / 64;
    for (uint64_t i = 0; i < full; i++) compress(st, msg + 64 * i);
    uint8_t tail[128];
    uint64_t rem = len - 64 * full;
    memset(tail, 0, sizeof tail);
    if (rem) memcpy(tail, msg + 64 * full, (size_t)rem);
    tail[rem] = 0x80;
    uint64_t tl = (rem + 9 <= 64) ? 64 : 128;
    uint64_t bits = len * 8;
    for (int i = 0; i < 8; i++) tail[tl - 1 - i] = (uint8_t)(bits >> (8 * i));
    compress(st, tail);
    if (tl == 128) compress(st, tail + 64);
}

void hdrf_oracle_sha1(const uint8_t *msg, uint64_t len, uint8_t out[20])
{
    uint32_t st[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    md_hash(msg, len, st, (void (*)(uint32_t *, const uint8_t *))sha1_compress);
    for (int i = 0; i < 20; i++) out[i] = (uint8_t)(st[i / 4] >> (24 - 8 * (i % 4)));
}

void hdrf_oracle_sha224(const uint8_t *msg, uint64_t len, uint8_t out[28])
{
    uint32_t st[8] = {0xc1059ed8u, 0x367cd507u, 0x3070dd17u, 0xf70e5939u,
                      0xffc00b31u, 0x68581511u, 0x64f98fa7u, 0xbefa4fa4u};
    md_hash(msg, len, st, (void (*)(uint32_t *, const uint8_t *))sha256_compress);
    for (int i = 0; i < 28; i++) out[i] = (uint8_t)(st[i / 4] >> (24 - 8 * (i % 4)));
}

/* ------------------------------------------------------------------------------------------ */
/* Redis restatement: a GET/SET map keyed by digest bytes (fixed length H) with 11-byte values. */
typedef struct {
    uint8_t *keys;    /* cap * H */
    uint8_t *vals;    /* cap * 11 */
    uint8_t *used;    /* cap */
    int64_t cap, count;
    int H;
} kvmap;

static uint64_t key_hash(const uint8_t *k, int H)
{
    uint64_t h = 1469598103934665603ull;
    for (int i = 0; i < H; i++) { h ^= k[i]; h *= 1099511628211ull; }
    return h ^ (h >> 29);
}

static int kv_init(kvmap *m, int H, int64_t cap)
{
    m->H = H; m->cap = cap; m->count = 0;
    m->keys = (uint8_t *)calloc((size_t)cap, (size_t)H);
    m->vals = (uint8_t *)calloc((size_t)cap, 11);
    m->used = (uint8_t *)calloc((size_t)cap, 1);
    return (m->keys && m->vals && m->used) ? 0 : -1;
}

static void kv_free(kvmap *m) { free(m->keys); free(m->vals); free(m->used); }

static int64_t kv_find(const kvmap *m, const uint8_t *k)
{
    uint64_t i = key_hash(k, m->H) & (uint64_t)(m->cap - 1);
    while (m->used[i]) {
        if (memcmp(m->keys + i * m->H, k, (size_t)m->H) == 0) return (int64_t)i;
        i = (i + 1) & (uint64_t)(m->cap - 1);
    }
    return -1 - (int64_t)i;
}

static int kv_set(kvmap *m, const uint8_t *k, const uint8_t *v11);

static int kv_grow(kvmap *m)
{
    kvmap n;
    if (kv_init(&n, m->H, m->cap * 2)) return -1;
    for (int64_t i = 0; i < m->cap; i++)
        if (m->used[i]) kv_set(&n, m->keys + i * m->H, m->vals + i * 11);
    kv_free(m);
    *m = n;
    return 0;
}

static int kv_set(kvmap *m, const uint8_t *k, const uint8_t *v11)
{
    if ((m->count + 1) * 2 > m->cap && kv_grow(m)) return -1;
    int64_t f = kv_find(m, k);
    int64_t i = f >= 0 ? f : -1 - f;
    if (f < 0) { m->used[i] = 1; memcpy(m->keys + i * m->H, k, (size_t)m->H); m->count++; }
    memcpy(m->vals + i * 11, v11, 11);
    return 0;
}

/* Container files (chunkDir + id): in-memory byte vectors keyed by 24-bit id. */
typedef struct {
    uint32_t id;
    uint8_t *data;
    int64_t len, cap;
    int closed;
    uint8_t *cdata;          /* compressor == 2: the file as rewritten on close (Lz4Codec stream) */
    int64_t clen;
} container;

/* Recipes: SET longToBytes(blockId,4) -> [BE32 size | digests] (DataDeduplicator.storeDB :372-392). */
typedef struct {
    uint32_t key;
    uint8_t *data;
    int64_t len;
} recipe;

struct hdrf_oracle {
    int hasher, compressor, H;
    uint32_t max_size;
    kvmap index;
    int have_alloc;
    uint8_t alloc[24];              /* Redis key "blockID" */
    /* one table per storer range (id >> 22): the range's storer thread is the only writer */
    container *cont[4]; int64_t ncont[4], ccap[4];
    recipe *rec; int64_t nrec, rcap;
    int mt_store;                   /* 1: the storer ranges run on concurrent threads (CPU baselines) */
    int store_only;                 /* 1: container and recipe BYTES are not kept (lengths, index values,
                                       allocator and storeSize are): bench.py's whole-corpus check */
};

hdrf_oracle *hdrf_oracle_new(int hasher, int compressor, uint32_t max_size)
{
    if (hasher != 0 && hasher != 1) return NULL;
    hdrf_oracle *o = (hdrf_oracle *)calloc(1, sizeof *o);
    if (!o) return NULL;
    o->hasher = hasher;
    o->compressor = compressor;
    o->H = hasher == 0 ? 20 : 28;                        /* DataNode.initializeDD :528-532 */
    o->max_size = max_size;                              /* DataDeduplicator.maxSize = 2^25 :434,527 */
    if (kv_init(&o->index, o->H, 1 << 16)) { free(o); return NULL; }
    return o;
}

void hdrf_oracle_set_store_only(hdrf_oracle *o, int on) { if (o) o->store_only = on != 0; }

void hdrf_oracle_free(hdrf_oracle *o)
{
    if (!o) return;
    kv_free(&o->index);
    for (int r = 0; r < 4; r++) {
        for (int64_t i = 0; i < o->ncont[r]; i++) { free(o->cont[r][i].data); free(o->cont[r][i].cdata); }
        free(o->cont[r]);
    }
    for (int64_t i = 0; i < o->nrec; i++) free(o->rec[i].data);
    free(o->rec); free(o);
}

static container *cont_find(const hdrf_oracle *o, uint32_t id)
{
    const int r = (int)(id >> 22) & 3;
    for (int64_t i = o->ncont[r] - 1; i >= 0; i--)
        if (o->cont[r][i].id == id) return &o->cont[r][i];
    return NULL;
}

static container *cont_create(hdrf_oracle *o, uint32_t id)
{
    const int r = (int)(id >> 22) & 3;
    if (o->ncont[r] == o->ccap[r]) {
        o->ccap[r] = o->ccap[r] ? o->ccap[r] * 2 : 16;
        o->cont[r] = (container *)realloc(o->cont[r], (size_t)o->ccap[r] * sizeof(container));
    }
    container *c = &o->cont[r][o->ncont[r]++];
    memset(c, 0, sizeof *c);
    c->id = id;
    return c;
}

static void cont_append(container *c, const uint8_t *p, int64_t n, int store_only)
{
    if (store_only) { c->len += n; return; }
    if (c->len + n > c->cap) {
        int64_t nc = c->cap ? c->cap : 4096;
        while (nc < c->len + n) nc *= 2;
        c->data = (uint8_t *)realloc(c->data, (size_t)nc);
        c->cap = nc;
    }
    memcpy(c->data + c->len, p, (size_t)n);
    c->len += n;
}

/* chunkMeta — DN/chunkMeta.java:7-87 */
typedef struct {
    int newChunk;
    int nCopy;
    int64_t blockID;
    int32_t blockStart, blockStop, bbStart, bbStop, length;
} chunk_meta;

/* chunkMeta.process(-1) — DN/chunkMeta.java:35-60 (decode an 11-byte Redis reply). */
static void meta_process(chunk_meta *c, const uint8_t *v /* NULL = nil reply */)
{
    if (!v) { c->newChunk = 1; c->nCopy = 1; return; }
    c->newChunk = 0;
    c->nCopy = v[0] & 0xFF;
    c->blockID = ((int64_t)v[1] << 16) | ((int64_t)v[2] << 8) | v[3];
    c->blockStart = (int32_t)(((uint32_t)(v[10] & 0xF0) << 20) | ((uint32_t)v[4] << 16) | ((uint32_t)v[5] << 8) | v[6]);
    c->blockStop = (int32_t)(((uint32_t)(v[10] & 0x0F) << 24) | ((uint32_t)v[7] << 16) | ((uint32_t)v[8] << 8) | v[9]);
    c->length = c->blockStop - c->blockStart;
    c->nCopy++;
}

/* chunkMeta.getMeta — DN/chunkMeta.java:62-77 (encode the 11-byte value). */
static void meta_encode(const chunk_meta *c, uint8_t v[11])
{
    v[0] = (uint8_t)c->nCopy;
    v[1] = (uint8_t)(c->blockID >> 16); v[2] = (uint8_t)(c->blockID >> 8); v[3] = (uint8_t)c->blockID;
    v[4] = (uint8_t)(c->blockStart >> 16); v[5] = (uint8_t)(c->blockStart >> 8); v[6] = (uint8_t)c->blockStart;
    v[7] = (uint8_t)(c->blockStop >> 16); v[8] = (uint8_t)(c->blockStop >> 8); v[9] = (uint8_t)c->blockStop;
    v[10] = (uint8_t)(((c->blockStart >> 20) & 0xF0) | ((c->blockStop >> 24) & 0x0F));
}

/* utilities.bytesToBlockID / bytesToBlockPos — DN/utilities.java:36-65 */
static int64_t bytes_to_slot(const uint8_t *b, int slot)
{
    return ((int64_t)b[slot * 3] << 16) | ((int64_t)b[slot * 3 + 1] << 8) | b[slot * 3 + 2];
}

/* DataDeduplicator(ByteBuffer, long) — DN/DataDeduplicator.java:108-217.
 * Blocks are processed in call order (the FIFO AIWriteQueue, :124-158,197-204). */
/* :122 chunking + :174 threadedHasher digests: the part of a block's reduction that does not
 * touch Redis (the reference runs it before the FIFO wait, DN/DataDeduplicator.java:122-124).
 * Returns n (off/dig malloc'ed, caller frees) or < 0. */
static int64_t chunk_and_hash(int hasher, int H, const uint8_t *data, int64_t size, uint32_t **off_out,
                              uint8_t **dig_out)
{
    int64_t ocap = size / 700 + 2;
    uint32_t *off = (uint32_t *)malloc((size_t)ocap * sizeof(uint32_t));
    if (!off) return -2;
    int64_t n = hdrf_oracle_chunk(data, size, off, ocap);
    if (n < 0) { free(off); return -1; }
    uint8_t *dig = (uint8_t *)malloc((size_t)n * H + 1);
    if (!dig) { free(off); return -2; }
    int64_t cur = 0;
    for (int64_t k = 0; k < n; k++) {
        if (hasher == 0) hdrf_oracle_sha1(data + cur, (uint64_t)(off[k] - cur), dig + k * H);
        else hdrf_oracle_sha224(data + cur, (uint64_t)(off[k] - cur), dig + k * H);
        cur = off[k];
    }
    *off_out = off;
    *dig_out = dig;
    return n;
}

static int64_t reduce_hashed(hdrf_oracle *o, const uint8_t *data, int64_t size, int64_t block_id, uint32_t *off,
                             int64_t n, uint8_t *dig, uint32_t *offsets_out, uint8_t *digests_out,
                             uint8_t *is_new_out, uint8_t *values_out, int64_t *store_size_out);

int64_t hdrf_oracle_reduce(hdrf_oracle *o, const uint8_t *data, int64_t size, int64_t block_id,
                           int64_t cap, uint32_t *offsets_out, uint8_t *digests_out, uint8_t *is_new_out,
                           uint8_t *values_out, int64_t *store_size_out)
{
    uint32_t *off = NULL;
    uint8_t *dig = NULL;
    int64_t n = chunk_and_hash(o->hasher, o->H, data, size, &off, &dig);
    if (n < 0) return n;
    if (n > cap) { free(off); free(dig); return -1; }
    return reduce_hashed(o, data, size, block_id, off, n, dig, offsets_out, digests_out, is_new_out, values_out,
                         store_size_out);
}

/* One threadedStorer (:702-836) over chunks [start, stop): appends the range's new chunks to its
 * container chain lastBlockID[t] (its own table of containers: the ranges never share one), closes
 * (and under compressor 2 compresses) a container when the next chunk would pass maxSize, and
 * encodes every chunk's value into setv. */
typedef struct {
    hdrf_oracle *o;
    const uint8_t *data;
    chunk_meta *cm;
    uint8_t *setv;
    int64_t start, stop, storeSize;
    int64_t *lastBlockID;
    int t;
} store_job;

static void *store_range(void *arg)
{
    store_job *j = (store_job *)arg;
    hdrf_oracle *o = j->o;
    chunk_meta *cm = j->cm;
    int64_t *lastBlockID = j->lastBlockID;
    const int t = j->t;
    if (j->storeSize == 0) {                                                /* :713-719 */
        for (int64_t k = j->start; k < j->stop; k++) meta_encode(&cm[k], j->setv + k * 11);
        return NULL;
    }
    container *c = cont_find(o, (uint32_t)lastBlockID[t]);                  /* :723-737 */
    int64_t curPos;
    if (c) curPos = c->len; else { c = cont_create(o, (uint32_t)lastBlockID[t]); curPos = 0; }
    int64_t bufpos = 0;                                                     /* bufferBB.position() */
    for (int64_t k = j->start; k < j->stop; k++) {
        if (cm[k].newChunk) {
            if (curPos + cm[k].length > (int64_t)o->max_size) {            /* :748 buffer full */
                c->closed = 1;                                              /* :754-786 rewrite prev||buf */
                if (o->compressor == 2 && !o->store_only) {                 /* :770-779 Lz4Codec stream */
                    c->cdata = (uint8_t *)malloc((size_t)hdrf_oracle_hadoop_lz4_bound(c->len));
                    c->clen = hdrf_oracle_hadoop_lz4_frame(c->data, c->len, c->cdata);
                }
                bufpos = 0; curPos = 0;                                     /* :790-791 */
                lastBlockID[t]++;                                           /* :792 */
                lastBlockID[t + 4] = 0;                                     /* :793 */
                c = cont_find(o, (uint32_t)lastBlockID[t]);                /* :794-795 createNewFile */
                if (!c) c = cont_create(o, (uint32_t)lastBlockID[t]);
            }
            cont_append(c, j->data + cm[k].bbStart, cm[k].length, o->store_only);   /* :798 */
            bufpos += cm[k].length;
            cm[k].blockID = lastBlockID[t];                                 /* :799 */
            cm[k].blockStart = (int32_t)curPos;                             /* :800 setBlockStartStop */
            cm[k].blockStop = (int32_t)(curPos + cm[k].length);
            curPos += cm[k].length;                                         /* :801 */
        }
        meta_encode(&cm[k], j->setv + k * 11);                              /* :803 SET digest -> meta */
    }
    lastBlockID[t + 4] = bufpos;                                            /* :808 */
    return NULL;
}

/* The ordered part (FIFO turn, :124-204): Redis lookups, checkChunk, storers, SETs, storeDB.
 * Takes ownership of off/dig. */
static int64_t reduce_hashed(hdrf_oracle *o, const uint8_t *data, int64_t size, int64_t block_id, uint32_t *off,
                             int64_t n, uint8_t *dig, uint32_t *offsets_out, uint8_t *digests_out,
                             uint8_t *is_new_out, uint8_t *values_out, int64_t *store_size_out)
{
    const int H = o->H;

    /* :165-172 allocator: GET "blockID"; absent -> (t<<22, 0) */
    int64_t lastBlockID[8];
    for (int i = 0; i < 4; i++) {
        lastBlockID[i] = o->have_alloc ? bytes_to_slot(o->alloc, i) : ((int64_t)i << 22);
        lastBlockID[i + 4] = o->have_alloc ? bytes_to_slot(o->alloc, i + 4) : 0;
    }

    /* :174 chunkHash -> threadedHasher.run :578-641: hash every chunk, then the MULTI'd
     * GETs are all answered before any of this block's SETs (storers start afterwards). */
    chunk_meta *cm = (chunk_meta *)calloc((size_t)n, sizeof(chunk_meta));
    if (!cm) { free(off); free(dig); return -2; }
    int64_t cur = 0;
    for (int64_t k = 0; k < n; k++) {
        int64_t end = off[k];
        cm[k].bbStart = (int32_t)cur; cm[k].bbStop = (int32_t)end; cm[k].length = (int32_t)(end - cur);
        int64_t f = kv_find(&o->index, dig + k * H);
        meta_process(&cm[k], f >= 0 ? o->index.vals + f * 11 : NULL);
        cur = end;
    }

    /* :178 checkChunk :338-367 — identity-keyed HashMap: every chunk takes the else branch,
     * so the only effect is storeSize = sum of new-chunk lengths. */
    int64_t storeSize = 0;
    for (int64_t k = 0; k < n; k++) if (cm[k].newChunk) storeSize += cm[k].length;

    /* :184 storeChunksMT :511-532 -> threadedStorer.run :702-836 */
    int nThread = n < 25 ? 1 : 3;
    uint8_t *setv = (uint8_t *)malloc((size_t)n * 11 + 1);
    store_job sj[3];
    pthread_t sth[3];
    int sstarted[3] = {0, 0, 0};
    for (int t = 0; t < nThread; t++) {
        sj[t] = (store_job){o, data, cm, setv, n * t / nThread, n * (t + 1) / nThread, storeSize, lastBlockID, t};
        /* the reference runs the ranges on three threadedStorer threads (:676-697), each closing and
         * compressing its own containers; the CPU baselines do too (o->mt_store) */
        if (o->mt_store && nThread > 1) sstarted[t] = pthread_create(&sth[t], NULL, store_range, &sj[t]) == 0;
        if (!sstarted[t]) store_range(&sj[t]);
    }
    for (int t = 0; t < nThread; t++)
        if (sstarted[t]) pthread_join(sth[t], NULL);
    /* Pipelined SETs: thread 0's, then thread 1's, then thread 2's (each in chunk order).
     * Cross-thread order is racy in the reference; this fixes "last occurrence in chunk order wins". */
    for (int64_t k = 0; k < n; k++) kv_set(&o->index, dig + k * H, setv + k * 11);

    /* :190 storeDB :372-392 (store_only: the allocator, no recipe bytes) */
    for (int i = 0; i < 8; i++) {                                           /* utilities.blockIDtoBytes :66-75 */
        o->alloc[i * 3] = (uint8_t)(lastBlockID[i] >> 16);
        o->alloc[i * 3 + 1] = (uint8_t)(lastBlockID[i] >> 8);
        o->alloc[i * 3 + 2] = (uint8_t)lastBlockID[i];
    }
    o->have_alloc = 1;
    uint32_t rkey = (uint32_t)block_id;                                     /* longToBytes(filename,4) */
    recipe *r = NULL;
    if (!o->store_only)
        for (int64_t i = 0; i < o->nrec; i++) if (o->rec[i].key == rkey) r = &o->rec[i];
    if (!r && !o->store_only) {
        if (o->nrec == o->rcap) {
            o->rcap = o->rcap ? o->rcap * 2 : 16;
            o->rec = (recipe *)realloc(o->rec, (size_t)o->rcap * sizeof(recipe));
        }
        r = &o->rec[o->nrec++];
        r->key = rkey; r->data = NULL;
    }
    if (r) {
        free(r->data);
        r->len = 4 + n * H;
        r->data = (uint8_t *)malloc((size_t)r->len);
        r->data[0] = (uint8_t)(size >> 24); r->data[1] = (uint8_t)(size >> 16);
        r->data[2] = (uint8_t)(size >> 8);  r->data[3] = (uint8_t)size;
        memcpy(r->data + 4, dig, (size_t)(n * H));
    }

    if (offsets_out) memcpy(offsets_out, off, (size_t)n * sizeof(uint32_t));
    if (digests_out) memcpy(digests_out, dig, (size_t)(n * H));
    if (is_new_out) for (int64_t k = 0; k < n; k++) is_new_out[k] = (uint8_t)cm[k].newChunk;
    if (values_out) memcpy(values_out, setv, (size_t)n * 11);
    if (store_size_out) *store_size_out = storeSize;
    free(off); free(cm); free(dig); free(setv);
    return n;
}

/* ---- threaded CPU baseline (bench.py cpu_baseline only; never a checker) ------------------
 * The reference's concurrency shape: chunking + hashing of a block run before its FIFO turn
 * (DN/DataDeduplicator.java:122-124), so worker threads chunk and hash blocks ahead while the
 * ordered part (Redis lookups, checkChunk, storers, storeDB) takes the blocks one at a time in
 * arrival order (:124-204).  Results are those of hdrf_oracle_reduce called in order. */
typedef struct {
    const uint8_t *data;
    int64_t size;
    uint32_t *off;
    uint8_t *dig;
    int64_t n;
    int ready;
} hash_job;

typedef struct {
    hash_job *jobs;
    int64_t njobs;
    int64_t next;          /* next job to take (atomic) */
    int64_t consumed;      /* jobs the ordered part finished (atomic): bounds the lookahead */
    int64_t ahead;
    int hasher, H;
} hash_pool;

static void *hash_worker(void *arg)
{
    hash_pool *p = (hash_pool *)arg;
    for (;;) {
        const int64_t i = __atomic_fetch_add(&p->next, 1, __ATOMIC_RELAXED);
        if (i >= p->njobs) return NULL;
        while (i - __atomic_load_n(&p->consumed, __ATOMIC_ACQUIRE) > p->ahead) sched_yield();
        hash_job *j = &p->jobs[i];
        j->n = chunk_and_hash(p->hasher, p->H, j->data, j->size, &j->off, &j->dig);
        __atomic_store_n(&j->ready, 1, __ATOMIC_RELEASE);
    }
}

int64_t hdrf_oracle_reduce_many(hdrf_oracle *o, const uint8_t *const *blocks, const int64_t *sizes,
                                const int64_t *ids, int64_t nblocks, int nthreads, int64_t *store_sizes)
{
    return hdrf_oracle_reduce_many_out(o, blocks, sizes, ids, nblocks, nthreads, store_sizes, NULL, NULL);
}

/* The same with every block's full result (the parity tests at the bench's batch shape):
 * out[i] (may be NULL) receives what hdrf_oracle_reduce would write for block i, and
 * counts[i] its chunk count; out[i].cap bounds the chunk arrays (-1 past it). */
int64_t hdrf_oracle_reduce_many_out(hdrf_oracle *o, const uint8_t *const *blocks, const int64_t *sizes,
                                    const int64_t *ids, int64_t nblocks, int nthreads, int64_t *store_sizes,
                                    const hdrf_oracle_out *out, int64_t *counts)
{
    if (nthreads < 1) nthreads = 1;
    o->mt_store = 1;                     /* CPU baseline: three concurrent storers per block */
    hash_pool p;
    memset(&p, 0, sizeof p);
    p.jobs = (hash_job *)calloc((size_t)(nblocks > 0 ? nblocks : 1), sizeof(hash_job));
    if (!p.jobs) return -2;
    p.njobs = nblocks; p.ahead = 2 * nthreads; p.hasher = o->hasher; p.H = o->H;
    for (int64_t i = 0; i < nblocks; i++) { p.jobs[i].data = blocks[i]; p.jobs[i].size = sizes[i]; }
    pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    int started = 0;
    for (int t = 0; t < nthreads; t++)
        if (pthread_create(&th[t], NULL, hash_worker, &p) == 0) started++;
    int64_t rc = 0;
    if (!started) rc = -2;
    for (int64_t i = 0; i < nblocks && rc >= 0; i++) {
        hash_job *j = &p.jobs[i];
        while (!__atomic_load_n(&j->ready, __ATOMIC_ACQUIRE)) sched_yield();
        if (j->n < 0) { rc = j->n; break; }
        int64_t ss = 0;
        const hdrf_oracle_out *w = out ? &out[i] : NULL;
        if (w && j->n > w->cap) { rc = -1; break; }
        const int64_t n = reduce_hashed(o, j->data, j->size, ids[i], j->off, j->n, j->dig, w ? w->offsets : NULL,
                                        w ? w->digests : NULL, w ? w->is_new : NULL, w ? w->values : NULL, &ss);
        j->off = NULL; j->dig = NULL;
        if (counts) counts[i] = n;
        if (n < 0) { rc = n; break; }
        if (store_sizes) store_sizes[i] = ss;
        __atomic_store_n(&p.consumed, i + 1, __ATOMIC_RELEASE);
    }
    __atomic_store_n(&p.consumed, nblocks + p.ahead + 1, __ATOMIC_RELEASE);   /* release waiting workers */
    for (int t = 0; t < nthreads; t++)
        if (t < started) pthread_join(th[t], NULL);
    for (int64_t i = 0; i < nblocks; i++) { free(p.jobs[i].off); free(p.jobs[i].dig); }
    free(th);
    free(p.jobs);
    o->mt_store = 0;
    return rc < 0 ? rc : nblocks;
}

/* The reference's own concurrency shape, blocks serialised (BASELINE.md CPU plan 1): per block
 * chunking on one thread (DN/DataDeduplicator.java:122), then nhash threadedHasher threads over
 * the chunk ranges [n*t/nhash, n*(t+1)/nhash) (:168-185, :578-641), then the ordered part on the
 * calling thread (Redis lookups, checkChunk, storers, storeDB).  The reference's 3 storer threads
 * copy into 3 different containers; here those appends run on the calling thread (a memcpy share
 * of the block's time well under its hashing).  Results equal hdrf_oracle_reduce in order. */
typedef struct {
    int hasher, H;
    const uint8_t *data;
    const uint32_t *off;
    uint8_t *dig;
    int64_t k0, k1;
} hash_range;

static void *hash_range_worker(void *arg)
{
    hash_range *r = (hash_range *)arg;
    int64_t cur = r->k0 ? r->off[r->k0 - 1] : 0;
    for (int64_t k = r->k0; k < r->k1; k++) {
        if (r->hasher == 0) hdrf_oracle_sha1(r->data + cur, (uint64_t)(r->off[k] - cur), r->dig + k * r->H);
        else hdrf_oracle_sha224(r->data + cur, (uint64_t)(r->off[k] - cur), r->dig + k * r->H);
        cur = r->off[k];
    }
    return NULL;
}

int64_t hdrf_oracle_reduce_ref_shape(hdrf_oracle *o, const uint8_t *const *blocks, const int64_t *sizes,
                                     const int64_t *ids, int64_t nblocks, int nhash, int64_t *store_sizes)
{
    if (nhash < 1) nhash = 1;
    if (nhash > 64) nhash = 64;
    o->mt_store = 1;                     /* the three threadedStorer threads (:676-697) run at once */
    int64_t rc = nblocks;
    for (int64_t i = 0; i < nblocks && rc >= 0; i++) {
        const int64_t ocap = sizes[i] / 700 + 2;
        uint32_t *off = (uint32_t *)malloc((size_t)ocap * sizeof(uint32_t));
        if (!off) { rc = -2; break; }
        const int64_t n = hdrf_oracle_chunk(blocks[i], sizes[i], off, ocap);
        if (n < 0) { free(off); rc = -1; break; }
        uint8_t *dig = (uint8_t *)malloc((size_t)n * o->H + 1);
        if (!dig) { free(off); rc = -2; break; }
        pthread_t th[64];
        hash_range rg[64];
        int started[64] = {0};
        for (int t = 0; t < nhash; t++) {
            rg[t].hasher = o->hasher; rg[t].H = o->H; rg[t].data = blocks[i]; rg[t].off = off; rg[t].dig = dig;
            rg[t].k0 = n * t / nhash; rg[t].k1 = n * (t + 1) / nhash;
            started[t] = pthread_create(&th[t], NULL, hash_range_worker, &rg[t]) == 0;
            if (!started[t]) hash_range_worker(&rg[t]);
        }
        for (int t = 0; t < nhash; t++)
            if (started[t]) pthread_join(th[t], NULL);
        int64_t ss = 0;
        const int64_t r = reduce_hashed(o, blocks[i], sizes[i], ids[i], off, n, dig, NULL, NULL, NULL, NULL, &ss);
        if (r < 0) { rc = r; break; }
        if (store_sizes) store_sizes[i] = ss;
    }
    o->mt_store = 0;
    return rc;
}

int hdrf_oracle_index_get(const hdrf_oracle *o, const uint8_t *digest, uint8_t out11[11])
{
    int64_t f = kv_find(&o->index, digest);
    if (f < 0) return 0;
    memcpy(out11, o->index.vals + f * 11, 11);
    return 1;
}

int64_t hdrf_oracle_index_count(const hdrf_oracle *o) { return o->index.count; }

static int g_sort_H;
static int cmp_keyidx(const void *a, const void *b)
{
    const uint8_t *const *pa = (const uint8_t *const *)a, *const *pb = (const uint8_t *const *)b;
    return memcmp(*pa, *pb, (size_t)g_sort_H);
}

int64_t hdrf_oracle_index_dump(const hdrf_oracle *o, uint8_t *keys, uint8_t *vals, int64_t cap)
{
    const kvmap *m = &o->index;
    if (cap < m->count) return -m->count;
    const uint8_t **ptr = (const uint8_t **)malloc((size_t)(m->count + 1) * sizeof(uint8_t *));
    int64_t j = 0;
    for (int64_t i = 0; i < m->cap; i++) if (m->used[i]) ptr[j++] = m->keys + i * m->H;
    g_sort_H = m->H;
    qsort(ptr, (size_t)j, sizeof(uint8_t *), cmp_keyidx);
    for (int64_t i = 0; i < j; i++) {
        int64_t slot = (ptr[i] - m->keys) / m->H;
        memcpy(keys + i * m->H, ptr[i], (size_t)m->H);
        memcpy(vals + i * 11, m->vals + slot * 11, 11);
    }
    free(ptr);
    return j;
}

int hdrf_oracle_allocator(const hdrf_oracle *o, uint8_t out24[24])
{
    if (!o->have_alloc) return 0;
    memcpy(out24, o->alloc, 24);
    return 1;
}

int64_t hdrf_oracle_recipe(const hdrf_oracle *o, int64_t block_id, uint8_t *out, int64_t cap)
{
    for (int64_t i = 0; i < o->nrec; i++)
        if (o->rec[i].key == (uint32_t)block_id) {
            if (cap < o->rec[i].len) return -o->rec[i].len;
            memcpy(out, o->rec[i].data, (size_t)o->rec[i].len);
            return o->rec[i].len;
        }
    return 0;
}

int64_t hdrf_oracle_container(const hdrf_oracle *o, uint32_t id, uint8_t *out, int64_t cap, int *closed)
{
    const container *c = o->store_only ? NULL : cont_find(o, id);
    if (!c) return -1;
    if (closed) *closed = c->closed;
    const uint8_t *src = c->cdata ? c->cdata : c->data;   /* closed + compressor 2: the LZ4 file */
    const int64_t len = c->cdata ? c->clen : c->len;
    if (cap < len) return -(len + 2);
    if (len) memcpy(out, src, (size_t)len);
    return len;
}

/* ------------------------------------------------------------------------------------------ */
/* Synthetic corpus (BASELINE config 2; spec in DESIGN.md §Corpus). */
uint64_t hdrf_oracle_mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void hdrf_oracle_corpus_roots(uint64_t seed, uint32_t dup_ppm, int64_t nblocks, int64_t spb, uint32_t *roots)
{
    for (int64_t b = 0; b < nblocks; b++)
        for (int64_t s = 0; s < spb; s++) {
            uint64_t g = (uint64_t)(b * spb + s);
            uint64_t coin = hdrf_oracle_mix64(seed ^ 0xD1B54A32D192ED03ull ^ hdrf_oracle_mix64(g));
            if (b > 0 && (coin % 1000000ull) < dup_ppm) {
                uint64_t r1 = hdrf_oracle_mix64(coin);
                uint64_t sb = r1 % (uint64_t)b;
                uint64_t ss = hdrf_oracle_mix64(r1) % (uint64_t)spb;
                roots[g] = roots[sb * spb + ss];
            } else {
                roots[g] = (uint32_t)g;
            }
        }
}

void hdrf_oracle_corpus_fill(uint64_t seed, const uint32_t *roots, int64_t block, int64_t spb,
                             int64_t seg_bytes, uint8_t *out)
{
    for (int64_t s = 0; s < spb; s++) {
        uint64_t key = hdrf_oracle_mix64(seed ^ hdrf_oracle_mix64((uint64_t)roots[block * spb + s] + 1));
        uint8_t *dst = out + s * seg_bytes;
        for (int64_t wi = 0; wi < seg_bytes / 8; wi++) {
            uint64_t x = hdrf_oracle_mix64(key + (uint64_t)wi);
            memcpy(dst + 8 * wi, &x, 8);            /* little-endian host */
        }
    }
}

/* java.util.Random — seed scramble, 48-bit LCG, nextInt(), nextBytes() (JDK 8 semantics). */
void hdrf_oracle_java_random_bytes(int64_t seed, int32_t buffer_len, int64_t total, uint8_t *out)
{
    uint64_t s = ((uint64_t)seed ^ 0x5DEECE66Dull) & ((1ull << 48) - 1);
    int64_t written = 0;
    while (written < total) {
        /* rb.nextBytes(toWrite): buffer_len bytes from ceil(buffer_len/4) nextInt() calls */
        for (int32_t i = 0; i < buffer_len;) {
            s = (s * 0x5DEECE66Dull + 0xBull) & ((1ull << 48) - 1);
            int32_t rnd = (int32_t)(uint32_t)(s >> 16);
            for (int nb = (buffer_len - i) < 4 ? (buffer_len - i) : 4; nb-- > 0; rnd >>= 8) {
                if (written + i < total) out[written + i] = (uint8_t)rnd;
                i++;
            }
        }
        written += buffer_len;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Compression stage (compressor == 2): Hadoop Lz4Codec over a closed container,
 * DN/DataDeduplicator.java:770-779 (codec.createOutputStream(output).write(temp); close()).
 *
 * Third-party algorithm, NOT under /root/reference (hadoop-common 3.1.0 is not vendored):
 *  - framing: org.apache.hadoop.io.compress.BlockCompressorStream with Lz4Codec's buffer size
 *    io.compression.codec.lz4.buffersize = 256 KiB, overhead 256 KiB/255 + 16, so
 *    MAX_INPUT_SIZE = 261,100; one write(temp) + close() gives
 *      len == 0            : BE32 0
 *      len <= 261,100      : BE32 len | BE32 clen | block
 *      len  > 261,100      : BE32 len | (BE32 clen | block) per 261,100-B segment | BE32 0
 *  - block: lz4 r123 LZ4_compress() (hadoop-common native Lz4Compressor.c), restated below.
 * Hadoop and r123 are not present here.  The restatement is pinned against a real liblz4 (the one
 * pyarrow 25.0.0 bundles, >= 1.9): run under the three rules where liblz4 >= 1.9 parses
 * differently from r123 (lz4_compress_rules below) it equals liblz4's LZ4_compress_default byte
 * for byte on every input tests/test_lz4_liblz4.py tries, and its r123 output decodes through
 * liblz4's decoder; the three r123 rules themselves are restated, not pinned.  The GPU must equal
 * the r123-rule output byte for byte. */
#define LZ4_MINMATCH 4
#define LZ4_MFLIMIT 12
#define LZ4_LASTLITERALS 5
#define LZ4_MAXDIST 65535
#define LZ4_SKIPSTRENGTH 6
#define LZ4_64KLIMIT (65536 + LZ4_MFLIMIT - 1)
#define LZ4_RUN_MASK 15
#define LZ4_ML_MASK 15
#define HADOOP_LZ4_MAX_INPUT 261100

static uint32_t lz_rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static int max_i(int a, int b) { return a > b ? a : b; }
static uint32_t lz_hash5(const uint8_t *p)              /* liblz4 >= 1.9 LZ4_hash5, byU32, little endian */
{
    uint64_t v;
    memcpy(&v, p, 8);
    return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - 12));
}

int64_t hdrf_oracle_lz4_bound(int64_t n) { return n + n / 255 + 16; }

/* LZ4_compress_generic(noDict, notLimited, byU16 when n < 64 KiB + 11 else byU32).
 *
 * `rules` (test infrastructure only, never r123): the three places where liblz4 >= 1.9 on a 64-bit
 * host parses differently from r123, so that the same restatement can be compared byte for byte
 * with a modern liblz4 (pyarrow's bundled one, tests/test_lz4_liblz4.py):
 *   bit 0  the search steps: 1, then searchMatchNb++ >> skipTrigger from 1 << skipTrigger, so
 *          step k is (63 + k) >> 6 (r123: (67 + k) >> 6, growing 4 attempts earlier);
 *   bit 1  the search gives up when the next position passes mflimit + 1 (r123: mflimit);
 *   bit 2  byU32 tables hash 5 bytes, ((v64 << 24) * 889523592379) >> (64 - 12) (r123: 4 bytes).
 * Everything else — table fill, catch-up, the test of the next position, token / length / offset
 * coding, last literals — is the shared code, which is what the comparison pins. */
static int64_t lz4_compress_rules(const uint8_t *src, int64_t n, uint8_t *dst, int rules)
{
    const int hlog = n < LZ4_64KLIMIT ? 13 : 12;           /* LZ4_HASHLOG(+1 for byU16), MEMORY_USAGE 14 */
    const int hash5 = (rules & 4) && n >= LZ4_64KLIMIT;
    uint32_t *table = (uint32_t *)calloc((size_t)1 << hlog, sizeof(uint32_t));
    const uint8_t *ip = src, *anchor = src;
    const uint8_t *const iend = src + n, *const mflimit = iend - LZ4_MFLIMIT, *const matchlimit = iend - LZ4_LASTLITERALS;
    const uint8_t *const slimit = (rules & 2) ? mflimit + 1 : mflimit;
    uint8_t *op = dst;
#define LZH(p) (hash5 ? lz_hash5(p) : (uint32_t)(lz_rd32(p) * 2654435761u) >> (32 - hlog))
    if (n >= LZ4_MFLIMIT + 1) {                            /* LZ4_minLength */
        table[LZH(ip)] = 0;                                /* first byte */
        ip++;
        uint32_t fh = LZH(ip);
        for (;;) {
            int attempts = (1 << LZ4_SKIPSTRENGTH) + ((rules & 1) ? -1 : 3);
            const uint8_t *fip = ip, *ref;
            uint8_t *token;
            do {                                           /* find a match */
                const uint32_t h = fh;
                const int step = max_i(1, attempts++ >> LZ4_SKIPSTRENGTH);
                ip = fip;
                fip = ip + step;
                if (fip > slimit) goto last_literals;
                fh = LZH(fip);
                ref = src + table[h];
                table[h] = (uint32_t)(ip - src);
            } while (ref + LZ4_MAXDIST < ip || lz_rd32(ref) != lz_rd32(ip));
            while (ip > anchor && ref > src && ip[-1] == ref[-1]) { ip--; ref--; }   /* catch up */
            {                                              /* literal length + literals */
                int64_t len = ip - anchor;
                token = op++;
                if (len >= LZ4_RUN_MASK) {
                    int64_t l = len - LZ4_RUN_MASK;
                    *token = LZ4_RUN_MASK << 4;
                    for (; l >= 255; l -= 255) *op++ = 255;
                    *op++ = (uint8_t)l;
                } else {
                    *token = (uint8_t)(len << 4);
                }
                memcpy(op, anchor, (size_t)len);
                op += len;
            }
        next_match:
            *op++ = (uint8_t)(ip - ref);                   /* offset, little-endian 16 */
            *op++ = (uint8_t)((ip - ref) >> 8);
            ip += LZ4_MINMATCH; ref += LZ4_MINMATCH;
            anchor = ip;
            while (ip < matchlimit && *ip == *ref) { ip++; ref++; }
            {
                int64_t len = ip - anchor;                 /* match length - 4 */
                if (len >= LZ4_ML_MASK) {
                    *token += LZ4_ML_MASK;
                    len -= LZ4_ML_MASK;
                    for (; len > 509; len -= 510) { *op++ = 255; *op++ = 255; }
                    if (len >= 255) { len -= 255; *op++ = 255; }
                    *op++ = (uint8_t)len;
                } else {
                    *token += (uint8_t)len;
                }
            }
            if (ip > mflimit) { anchor = ip; break; }      /* end of chunk */
            table[LZH(ip - 2)] = (uint32_t)(ip - 2 - src);  /* fill table */
            ref = src + table[LZH(ip)];                     /* test next position */
            table[LZH(ip)] = (uint32_t)(ip - src);
            if (ref + LZ4_MAXDIST >= ip && lz_rd32(ref) == lz_rd32(ip)) { token = op++; *token = 0; goto next_match; }
            anchor = ip++;
            fh = LZH(ip);
        }
    }
last_literals:
    {
        int64_t run = iend - anchor;
        if (run >= LZ4_RUN_MASK) {
            *op++ = LZ4_RUN_MASK << 4;
            run -= LZ4_RUN_MASK;
            for (; run >= 255; run -= 255) *op++ = 255;
            *op++ = (uint8_t)run;
        } else {
            *op++ = (uint8_t)(run << 4);
        }
        memcpy(op, anchor, (size_t)(iend - anchor));
        op += iend - anchor;
    }
#undef LZH
    free(table);
    return op - dst;
}

int64_t hdrf_oracle_lz4_compress(const uint8_t *src, int64_t n, uint8_t *dst) { return lz4_compress_rules(src, n, dst, 0); }

/* test infrastructure: the same parse under liblz4 >= 1.9's rules (above) */
int64_t hdrf_oracle_lz4_compress_modern(const uint8_t *src, int64_t n, uint8_t *dst, int rules)
{
    return lz4_compress_rules(src, n, dst, rules);
}

/* LZ4 block decoder (test helper; returns decoded length or -1 on malformed input) */
int64_t hdrf_oracle_lz4_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap)
{
    const uint8_t *ip = src, *const iend = src + n;
    int64_t o = 0;
    while (ip < iend) {
        const uint8_t tok = *ip++;
        int64_t lit = tok >> 4;
        if (lit == 15) { uint8_t b; do { if (ip >= iend) return -1; b = *ip++; lit += b; } while (b == 255); }
        if (ip + lit > iend || o + lit > cap) return -1;
        memcpy(dst + o, ip, (size_t)lit);
        ip += lit; o += lit;
        if (ip == iend) break;                               /* last literals */
        if (ip + 2 > iend) return -1;
        const int64_t off = ip[0] | (ip[1] << 8);
        ip += 2;
        int64_t ml = tok & 15;
        if (ml == 15) { uint8_t b; do { if (ip >= iend) return -1; b = *ip++; ml += b; } while (b == 255); }
        ml += 4;
        if (off == 0 || off > o || o + ml > cap) return -1;
        for (int64_t i = 0; i < ml; i++) dst[o + i] = dst[o - off + i];
        o += ml;
    }
    return o;
}

static uint8_t *put_be32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24); p[1] = (uint8_t)(v >> 16); p[2] = (uint8_t)(v >> 8); p[3] = (uint8_t)v;
    return p + 4;
}

int64_t hdrf_oracle_hadoop_lz4_bound(int64_t n)
{
    const int64_t nseg = n / HADOOP_LZ4_MAX_INPUT + 1;
    return 8 + nseg * 4 + hdrf_oracle_lz4_bound(n) + nseg * 16;
}

/* BlockCompressorStream(Lz4Compressor, 256 KiB).write(src, 0, n); close() */
int64_t hdrf_oracle_hadoop_lz4_frame(const uint8_t *src, int64_t n, uint8_t *dst)
{
    uint8_t *p = dst;
    if (n == 0) return put_be32(p, 0) - dst;
    p = put_be32(p, (uint32_t)n);
    for (int64_t off = 0; off < n; off += HADOOP_LZ4_MAX_INPUT) {
        const int64_t len = n - off < HADOOP_LZ4_MAX_INPUT ? n - off : HADOOP_LZ4_MAX_INPUT;
        const int64_t c = hdrf_oracle_lz4_compress(src + off, len, p + 4);
        put_be32(p, (uint32_t)c);
        p += 4 + c;
    }
    if (n > HADOOP_LZ4_MAX_INPUT) p = put_be32(p, 0);
    return p - dst;
}

/* Stream mode: BlockCompressorStream.write(b, off, len) per packet (hadoop-common 3.1.0
 * BlockCompressorStream.java, Lz4Compressor with its 256 KiB buffer):
 *   limlen = bytes buffered since the last reset
 *   if (len + limlen > MAX_INPUT && limlen > 0) { finish(); reset(); }
 *   if (len > MAX_INPUT) { BE32 len; per <= MAX_INPUT piece: BE32 clen, LZ4 block; reset() }
 *   else buffer (the 262,144-B buffer cannot fill below MAX_INPUT, so needsInput() stays true)
 * finish() = BE32 limlen, BE32 clen, LZ4 block of the buffered bytes; close() = finish(), which
 * writes BE32 0 when nothing is buffered (empty block, or a big write last). */
int64_t hdrf_oracle_hadoop_lz4_stream_bound(int64_t n, int64_t nwrites)
{
    return hdrf_oracle_hadoop_lz4_bound(n) + 24 * (nwrites + 1) + 16 * (n / HADOOP_LZ4_MAX_INPUT + 1);
}

static uint8_t *lz4_group(uint8_t *p, const uint8_t *src, int64_t n)
{
    p = put_be32(p, (uint32_t)n);
    const int64_t c = hdrf_oracle_lz4_compress(src, n, p + 4);
    put_be32(p, (uint32_t)c);
    return p + 4 + c;
}

int64_t hdrf_oracle_hadoop_lz4_stream(const uint8_t *src, const int64_t *writes, int64_t nwrites, uint8_t *dst)
{
    uint8_t *p = dst;
    int64_t off = 0, gs = 0, lim = 0;
    for (int64_t w = 0; w < nwrites; w++) {
        const int64_t len = writes[w];
        if (lim > 0 && len + lim > HADOOP_LZ4_MAX_INPUT) {      /* finish(); compressor.reset() */
            p = lz4_group(p, src + gs, lim);
            lim = 0;
        }
        if (len > HADOOP_LZ4_MAX_INPUT) {                         /* segmented write */
            p = put_be32(p, (uint32_t)len);
            for (int64_t o = 0; o < len; o += HADOOP_LZ4_MAX_INPUT) {
                const int64_t m = len - o < HADOOP_LZ4_MAX_INPUT ? len - o : HADOOP_LZ4_MAX_INPUT;
                const int64_t c = hdrf_oracle_lz4_compress(src + off + o, m, p + 4);
                put_be32(p, (uint32_t)c);
                p += 4 + c;
            }
            off += len;
            continue;
        }
        if (lim == 0) gs = off;
        lim += len;
        off += len;
    }
    p = lim > 0 ? lz4_group(p, src + gs, lim) : put_be32(p, 0);   /* close() */
    return p - dst;
}

/* ---- Snappy (stream mode compressor == 0, DN/BlockReceiver.java:826-873,887-894) ----------
 * Hadoop SnappyCodec (hadoop-common 3.1.0): BlockCompressorStream with a 256 KiB buffer and
 * compressionOverhead = bufferSize / 6 + 32, so MAX_INPUT = 218,422; each group is one
 * snappy::RawCompress call made by the native SnappyCompressor (snappy-c snappy_compress).
 * Third-party and not in the reference tree.  Restated from google/snappy's published
 * compressor (default level 1): varint(n), then independent fragments of 64 KiB, each with a
 * fresh hash table of max(256, next pow2 >= fragment) u16 entries capped at 2^15, hash
 * ((v * 0x1e35a7bd) >> 17) & mask, the skip heuristic (step = skip++ >> 5 from 32), greedy copies
 * with the ip-1 / ip table refresh, 64-byte copy splitting (>= 68: 64, > 64: 60).  Pinned byte
 * for byte against the snappy bundled in pyarrow (tests/test_snappy.py); vs Hadoop's own
 * libsnappy UNPINNED (its version is the host's). */
#define SNAPPY_FRAG 65536
#define HADOOP_SNAPPY_MAX_INPUT 218422

static uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }

static uint8_t *sn_literal(uint8_t *op, const uint8_t *lit, int64_t len)
{
    const uint32_t n = (uint32_t)(len - 1);
    if (n < 60) {
        *op++ = (uint8_t)(n << 2);
    } else {
        int cnt = 0;
        for (uint32_t t = n; t; t >>= 8) cnt++;
        *op++ = (uint8_t)((59 + cnt) << 2);
        for (int k = 0; k < cnt; k++) *op++ = (uint8_t)(n >> (8 * k));
    }
    memcpy(op, lit, (size_t)len);
    return op + len;
}

static uint8_t *sn_copy64(uint8_t *op, uint32_t off, uint32_t len)
{
    if (len < 12 && off < 2048) {
        *op++ = (uint8_t)(1 | ((len - 4) << 2) | ((off >> 8) << 5));
        *op++ = (uint8_t)off;
    } else {
        *op++ = (uint8_t)(2 | ((len - 1) << 2));
        *op++ = (uint8_t)off;
        *op++ = (uint8_t)(off >> 8);
    }
    return op;
}

static uint8_t *sn_copy(uint8_t *op, uint32_t off, int64_t len)
{
    while (len >= 68) { op = sn_copy64(op, off, 64); len -= 64; }
    if (len > 64) { op = sn_copy64(op, off, 60); len -= 60; }
    return sn_copy64(op, off, (uint32_t)len);
}

static uint8_t *sn_fragment(const uint8_t *src, int64_t n, uint8_t *op, uint16_t *tab)
{
    uint32_t ts = 256;
    while (ts < (1u << 15) && ts < n) ts <<= 1;
    const uint32_t mask = ts - 1;
    memset(tab, 0, ts * sizeof(uint16_t));
#define SNH(v) ((((uint32_t)(v) * 0x1e35a7bdu) >> 17) & mask)
    int64_t ip = 0;
    if (n >= 15) {
        const int64_t lim = n - 15;
        for (;;) {
            const int64_t next_emit = ip++;
            uint32_t skip = 32;
            int64_t cand;
            for (;;) {                                         /* search with growing strides */
                const uint32_t h = SNH(ld32(src + ip));
                const uint32_t step = skip >> 5;
                skip += step;
                if (ip + step > lim) { ip = next_emit; goto remainder; }
                cand = tab[h];
                tab[h] = (uint16_t)ip;
                if (ld32(src + ip) == ld32(src + cand)) break;
                ip += step;
            }
            op = sn_literal(op, src + next_emit, ip - next_emit);
            for (;;) {                                         /* copies back to back */
                const int64_t base = ip;
                int64_t m = 4;
                while (ip + m < n && src[cand + m] == src[ip + m]) m++;
                ip += m;
                op = sn_copy(op, (uint32_t)(base - cand), m);
                if (ip >= lim) goto remainder;
                tab[SNH(ld32(src + ip - 1))] = (uint16_t)(ip - 1);
                const uint32_t h = SNH(ld32(src + ip));
                cand = tab[h];
                tab[h] = (uint16_t)ip;
                if (ld32(src + ip) != ld32(src + cand)) break;
            }
        }
    }
remainder:
    if (ip < n) op = sn_literal(op, src + ip, n - ip);
#undef SNH
    return op;
}

int64_t hdrf_oracle_snappy_bound(int64_t n) { return 32 + n + n / 6; }

int64_t hdrf_oracle_snappy_compress(const uint8_t *src, int64_t n, uint8_t *dst)
{
    static __thread uint16_t tab[1 << 15];
    uint8_t *op = dst;
    for (uint64_t v = (uint64_t)n; ; v >>= 7) {             /* varint32 of the raw length */
        if (v < 0x80) { *op++ = (uint8_t)v; break; }
        *op++ = (uint8_t)(v | 0x80);
    }
    for (int64_t o = 0; o < n; o += SNAPPY_FRAG)
        op = sn_fragment(src + o, n - o < SNAPPY_FRAG ? n - o : SNAPPY_FRAG, op, tab);
    return op - dst;
}

/* snappy::RawUncompress; returns the decoded length or -1 on malformed input */
int64_t hdrf_oracle_snappy_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap)
{
    int64_t i = 0, o = 0;
    uint64_t raw = 0;
    for (int sh = 0;; sh += 7) {
        if (i >= n || sh > 28) return -1;
        const uint8_t b = src[i++];
        raw |= (uint64_t)(b & 0x7f) << sh;
        if (!(b & 0x80)) break;
    }
    if ((int64_t)raw > cap) return -1;
    while (i < n) {
        const uint8_t tag = src[i++];
        int64_t len, off;
        if ((tag & 3) == 0) {
            len = (tag >> 2) + 1;
            if (len > 60) {
                const int cnt = (int)len - 60;
                if (i + cnt > n) return -1;
                len = 0;
                for (int k = 0; k < cnt; k++) len |= (int64_t)src[i + k] << (8 * k);
                len += 1;
                i += cnt;
            }
            if (i + len > n || o + len > (int64_t)raw) return -1;
            memcpy(dst + o, src + i, (size_t)len);
            i += len; o += len;
            continue;
        }
        if ((tag & 3) == 1) {
            if (i + 1 > n) return -1;
            len = 4 + ((tag >> 2) & 7);
            off = ((int64_t)(tag >> 5) << 8) | src[i];
            i += 1;
        } else if ((tag & 3) == 2) {
            if (i + 2 > n) return -1;
            len = (tag >> 2) + 1;
            off = src[i] | ((int64_t)src[i + 1] << 8);
            i += 2;
        } else {
            if (i + 4 > n) return -1;
            len = (tag >> 2) + 1;
            off = (int64_t)ld32(src + i);
            i += 4;
        }
        if (off == 0 || off > o || o + len > (int64_t)raw) return -1;
        for (int64_t k = 0; k < len; k++) dst[o + k] = dst[o - off + k];
        o += len;
    }
    return o == (int64_t)raw ? o : -1;
}

/* Stream mode through a Hadoop BlockCompressorStream codec: 0 SnappyCodec, 4 Lz4Codec */
typedef int64_t (*raw_codec)(const uint8_t *, int64_t, uint8_t *);

static uint8_t *codec_group(uint8_t *p, const uint8_t *src, int64_t n, raw_codec f)
{
    p = put_be32(p, (uint32_t)n);
    const int64_t c = f(src, n, p + 4);
    put_be32(p, (uint32_t)c);
    return p + 4 + c;
}

int64_t hdrf_oracle_hadoop_stream_bound(int codec, int64_t n, int64_t nwrites)
{
    return codec == 0 ? hdrf_oracle_snappy_bound(n) + 24 * (nwrites + 1) + 48 * (n / HADOOP_SNAPPY_MAX_INPUT + 1)
                      : hdrf_oracle_hadoop_lz4_stream_bound(n, nwrites);
}

int64_t hdrf_oracle_hadoop_stream(int codec, const uint8_t *src, const int64_t *writes, int64_t nwrites, uint8_t *dst)
{
    if (codec == 4) return hdrf_oracle_hadoop_lz4_stream(src, writes, nwrites, dst);
    if (codec != 0) return -1;
    const raw_codec f = hdrf_oracle_snappy_compress;
    const int64_t MAX = HADOOP_SNAPPY_MAX_INPUT;
    uint8_t *p = dst;
    int64_t off = 0, gs = 0, lim = 0;
    for (int64_t w = 0; w < nwrites; w++) {
        const int64_t len = writes[w];
        if (lim > 0 && len + lim > MAX) { p = codec_group(p, src + gs, lim, f); lim = 0; }
        if (len > MAX) {
            p = put_be32(p, (uint32_t)len);
            for (int64_t o = 0; o < len; o += MAX) {
                const int64_t m = len - o < MAX ? len - o : MAX;
                const int64_t c = f(src + off + o, m, p + 4);
                put_be32(p, (uint32_t)c);
                p += 4 + c;
            }
            off += len;
            continue;
        }
        if (lim == 0) gs = off;
        lim += len;
        off += len;
    }
    p = lim > 0 ? codec_group(p, src + gs, lim, f) : put_be32(p, 0);
    return p - dst;
}

/* BlockDecompressorStream for codec 0 (snappy) or 4 (lz4); decoded length or -1 */
int64_t hdrf_oracle_hadoop_unframe(int codec, const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap)
{
    if (codec == 4) return hdrf_oracle_hadoop_lz4_unframe(src, n, dst, cap);
    if (codec != 0) return -1;
    int64_t o = 0, i = 0;
    while (i + 4 <= n) {
        const int64_t total = ((int64_t)src[i] << 24) | (src[i + 1] << 16) | (src[i + 2] << 8) | src[i + 3];
        i += 4;
        int64_t got = 0;
        while (got < total) {
            if (i + 4 > n) return -1;
            const int64_t c = ((int64_t)src[i] << 24) | (src[i + 1] << 16) | (src[i + 2] << 8) | src[i + 3];
            i += 4;
            if (i + c > n) return -1;
            const int64_t d = hdrf_oracle_snappy_decompress(src + i, c, dst + o, cap - o);
            if (d < 0) return -1;
            i += c; o += d; got += d;
        }
    }
    return i == n ? o : -1;
}

/* BlockDecompressorStream over the frame above; returns the decoded length or -1 */
int64_t hdrf_oracle_hadoop_lz4_unframe(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap)
{
    int64_t o = 0, i = 0;
    while (i + 4 <= n) {
        const int64_t total = ((int64_t)src[i] << 24) | (src[i + 1] << 16) | (src[i + 2] << 8) | src[i + 3];
        i += 4;
        int64_t got = 0;
        while (got < total) {
            if (i + 4 > n) return -1;
            const int64_t c = ((int64_t)src[i] << 24) | (src[i + 1] << 16) | (src[i + 2] << 8) | src[i + 3];
            i += 4;
            if (i + c > n) return -1;
            const int64_t d = hdrf_oracle_lz4_decompress(src + i, c, dst + o, cap - o);
            if (d < 0) return -1;
            i += c; o += d; got += d;
        }
    }
    return i == n ? o : -1;
}
