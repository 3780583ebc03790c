// inflate.hip — GzipCodec read side (DataNode.compressor 5) on gfx950: RFC 1951 inflate of a gzip
// member's deflate stream, plus the CRC-32 of the output.
//
// Reference: DN/DataConstructor.java:194-218 — a compressor-5 block file is read back through
// GzipCodec.createInputStream (Hadoop's DecompressorStream over zlib inflate, hadoop-common 3.1.0);
// tests check the output byte for byte against Python's zlib.decompress of the same file.
//
// A deflate stream is one sequential bit stream: a block's start is known only once the block
// before it is decoded.  A block file is one gzip member of up to 128 MiB, so one sequential
// decoder would serve a whole block at the speed of one wave.  Instead the member is cut into
// chunks of compressed bits and decoded speculatively, the way block-parallel CPU decompressors
// (pugz / rapidgzip, published) do it:
//   gz_find   one wave per chunk: the first bit offset in the chunk where a dynamic-Huffman block
//             header is valid (BTYPE 2, HLIT/HDIST in range, complete code-length code, the
//             code lengths decode within their counts, complete literal/length and distance
//             codes, a code for end-of-block) — a candidate block start.  Chunk 0 starts at bit 0.
//   gz_count  one wave per candidate: decode from the candidate, counting output, until a block
//             ends exactly at a later candidate (or the final block ends).  The host follows the
//             chain from chunk 0 (each link is a real block boundary, so false candidates are
//             never on it) and prefix-sums the counts.
//   gz_write  one wave per chunk on the chain: decode again into an LDS ring of 16-bit values —
//             bytes, or markers 256 + w for bytes of the 32 KiB window before the chunk that the
//             chunk cannot see yet — flushed to a u32 scratch at the chunk's output offset, the
//             markers as 256 + absolute source position.
//   gz_resolve  pointer jumping over the scratch until no marker is left (each pass replaces a
//             marker by what its source holds), then gz_pack narrows to bytes.
// The CRC-32 runs afterwards, one thread per 64 KiB piece (byte table in LDS); the host combines
// the piece CRCs (crc32_combine, zlib's published GF(2) method).
#include "bytes.hpp"
#include "launchers.hpp"

namespace hdrf {

constexpr int kInStage = 4096;               // staged compressed bytes (LDS)
constexpr int kRing = 32768;                 // u16 output ring = the deflate window
constexpr int kFlushAt = 16384;              // flush the ring every 16 Ki values
constexpr int kFastBits = 10;
constexpr int64_t kChunkBits = 8 * 32768;    // compressed bits per speculative chunk

struct HuffTab {
    uint16_t fast[1 << kFastBits];            // (len << 9) | symbol for codes <= 10 bits, 0 = slow path
    uint16_t count[16];                       // codes per length
    uint16_t sym[288];                        // symbols in canonical order
};

__constant__ uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2,
                                      3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193,
                                       257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145,
                                       8193, 12289, 16385, 24577};
__constant__ uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6,
                                       7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// Kraft check of n code lengths: 0 = complete, 1 = incomplete, -1 = over-subscribed
__device__ int kraft(const uint16_t *len, int n)
{
    int cnt[16] = {0};
    for (int s = 0; s < n; s++) cnt[len[s] & 15]++;
    int left = 1;
    for (int b = 1; b < 16; b++) {
        left = (left << 1) - cnt[b];
        if (left < 0) return -1;
    }
    return left > 0 ? 1 : 0;
}

// Decode tables from n code lengths (wave-cooperative).  false: not a code zlib's inflate accepts
// (over-subscribed, or incomplete with more than one code).
__device__ bool huff_build(HuffTab *t, const uint16_t *len, int n, bool dist)
{
    const int l = lane_id();
    __shared__ uint16_t offs_s[16];
    for (int i = l; i < (1 << kFastBits); i += 64) t->fast[i] = 0;
    if (l < 16) t->count[l] = 0;
    __syncthreads();
    bool ok = true;
    if (l == 0) {
        for (int s = 0; s < n; s++) t->count[len[s]]++;
        t->count[0] = 0;
        int left = 1, nz = 0;
        for (int b = 1; b < 16; b++) {
            left = (left << 1) - t->count[b];
            if (left < 0) ok = false;
            nz += t->count[b];
        }
        int maxl = 0;
        for (int b = 1; b < 16; b++)
            if (t->count[b]) maxl = b;
        if (ok && left > 0 && !(maxl == 1 || (dist && nz == 0))) ok = false;   // incomplete
        uint16_t o = 0;
        for (int b = 1; b < 16; b++) { offs_s[b] = o; o += t->count[b]; }
        for (int s = 0; s < n; s++)
            if (len[s]) t->sym[offs_s[len[s]]++] = (uint16_t)s;
        o = 0;
        for (int b = 1; b < 16; b++) { offs_s[b] = o; o += t->count[b]; }   // first sorted index per length
    }
    ok = __builtin_amdgcn_readfirstlane(ok ? 1 : 0) != 0;
    __syncthreads();
    // direct table: sorted symbol k of length b has canonical code first[b] + (k - offs[b]),
    // bit-reversed; it fills 2^(10-b) entries.  Lanes take sorted symbols.
    int first[16];
    {
        int code = 0;
        first[0] = 0;
        for (int b = 1; b < 16; b++) {
            code = (code + (b > 1 ? t->count[b - 1] : 0)) << 1;
            first[b] = code;
        }
    }
    int total = 0;
    for (int b = 1; b <= kFastBits; b++) total += t->count[b];
    for (int k = l; k < total; k += 64) {
        int b = 1;
        while (b < kFastBits && k >= offs_s[b] + t->count[b]) b++;
        const int code = first[b] + (k - offs_s[b]);
        const int r = (int)(__builtin_bitreverse32((uint32_t)code) >> (32 - b));
        const uint16_t e = (uint16_t)((b << 9) | t->sym[k]);
        for (int f = r; f < (1 << kFastBits); f += 1 << b) t->fast[f] = e;
    }
    __syncthreads();
    return ok;
}

// Bit reader over the compressed stream, staged in LDS; uniform state (scalar registers).
struct BitIn {
    const uint8_t *src;
    int64_t slen;
    uint32_t *stage;          // kInStage / 4 words of src[sbase, sbase + kInStage)
    int64_t sbase;
    int64_t nb;               // next (4-aligned) byte to pull
    uint64_t bb;
    int bn;

    __device__ __forceinline__ void restage(int64_t at)
    {
        const int l = lane_id();
        sbase = at & ~(int64_t)15;
        for (int k = 0; k < kInStage / 1024; k++) {
            const int64_t o = sbase + 16 * (l + 64 * k);
            uint4 v;
            if (o + 16 <= slen) v = ld16(src + o);
            else {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int i = 0; i < 16; i++)
                    if (o + i >= 0 && o + i < slen) w[i >> 2] |= (uint32_t)src[o + i] << (8 * (i & 3));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            *(uint4 *)(stage + 4 * (l + 64 * k)) = v;
        }
        __syncthreads();
    }
    __device__ __forceinline__ uint32_t word(int64_t at)     // 4 bytes at a 4-aligned offset
    {
        if (at < sbase || at + 4 > sbase + kInStage) restage(at);
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)stage[(at - sbase) >> 2]);
    }
    __device__ __forceinline__ void start(int64_t bit)
    {
        nb = (bit >> 3) & ~(int64_t)3;
        const int drop = (int)(bit - 8 * nb);
        bb = (uint64_t)word(nb) >> drop;
        bn = 32 - drop;
        nb += 4;
    }
    __device__ __forceinline__ void pull()
    {
        bb |= (uint64_t)word(nb) << bn;
        bn += 32;
        nb += 4;
    }
    __device__ __forceinline__ bool over() const { return nb > slen + 16; }   // decoding the zeros past the stream
    __device__ __forceinline__ uint32_t bits(int n)          // n <= 32
    {
        if (bn < n) pull();
        const uint32_t v = (uint32_t)(bb & ((n >= 32) ? 0xffffffffull : ((1ull << n) - 1)));
        bb >>= n;
        bn -= n;
        return v;
    }
    __device__ __forceinline__ int64_t pos() const { return 8 * nb - bn; }
    __device__ __forceinline__ int decode(const HuffTab *t)
    {
        if (bn < 32) pull();
        const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)t->fast[bb & ((1u << kFastBits) - 1)]);
        if (e) {
            const int n = (int)(e >> 9);
            bb >>= n;
            bn -= n;
            return (int)(e & 511);
        }
        int code = 0, first = 0, index = 0;
        for (int b = 1; b < 16; b++) {
            code |= (int)(bb & 1);
            bb >>= 1;
            bn--;
            const int count = t->count[b];
            if (code - count < first) return t->sym[index + (code - first)];
            index += count;
            first += count;
            first <<= 1;
            code <<= 1;
        }
        return -1;
    }
};

// Dynamic block header after BFINAL/BTYPE: the code lengths -> tables.  0 or < 0 (error)
// Kraft sum of n code lengths over the wave (sum of 2^(15 - len)); codes: number of nonzero lengths
__device__ __forceinline__ void kraft_wave(const uint16_t *len, int n, int &sum, int &codes, int &maxl)
{
    int s = 0, k = 0, m = 0;
    for (int i = lane_id(); i < n; i += 64) {
        const int v = len[i];
        if (v) { s += 1 << (15 - v); k++; m = max(m, v); }
    }
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o);
        k += __shfl_xor(k, o);
        m = max(m, __shfl_xor(m, o));
    }
    sum = s; codes = k; maxl = m;
}

template <bool kTables = true>
__device__ __forceinline__ int read_dynamic(BitIn &in, uint16_t *lens, HuffTab *hl, HuffTab *hd)
{
    const int l = lane_id();
    const int nlit = (int)in.bits(5) + 257, ndist = (int)in.bits(5) + 1, ncl = (int)in.bits(4) + 4;
    if (nlit > 286 || ndist > 30) return -4;
    for (int s = l; s < 19; s += 64) lens[s] = 0;
    __syncthreads();
    for (int i = 0; i < ncl; i++) {
        const uint32_t v = in.bits(3);
        if (l == 0) lens[kClOrder[i]] = (uint16_t)v;
    }
    __syncthreads();
    if (kraft(lens, 19) != 0) return -5;                 // the code-length code must be complete
    if (!huff_build(hl, lens, 19, false)) return -5;
    int i = 0;
    uint16_t prev = 0;
    while (i < nlit + ndist) {
        const int sym = in.decode(hl);
        if (sym < 0) return -6;
        int rep = 1;
        uint16_t v = (uint16_t)sym;
        if (sym == 16) { if (i == 0) return -7; v = prev; rep = 3 + (int)in.bits(2); }
        else if (sym == 17) { v = 0; rep = 3 + (int)in.bits(3); }
        else if (sym == 18) { v = 0; rep = 11 + (int)in.bits(7); }
        if (i + rep > nlit + ndist) return -8;
        __syncthreads();
        for (int k = l; k < rep; k += 64) lens[i + k] = v;
        __syncthreads();
        i += rep;
        prev = v;
    }
    if (lens[256] == 0) return -9;
    if (!kTables) {                                    // validation only (gz_find): zlib's rules
        int sum, codes, maxl;
        kraft_wave(lens, nlit, sum, codes, maxl);
        if (sum > (1 << 15) || (sum < (1 << 15) && maxl != 1)) return -10;
        kraft_wave(lens + nlit, ndist, sum, codes, maxl);
        if (sum > (1 << 15) || (sum < (1 << 15) && codes > 0 && maxl != 1)) return -10;
        return 0;
    }
    __syncthreads();
    const uint16_t dv = l < ndist ? lens[nlit + l] : 0;
    __syncthreads();
    if (l < 30) lens[288 + l] = l < ndist ? dv : 0;
    for (int s = nlit + l; s < 288; s += 64) lens[s] = 0;
    __syncthreads();
    if (!huff_build(hl, lens, 288, false)) return -10;
    if (!huff_build(hd, lens + 288, 30, true)) return -10;
    return 0;
}

__device__ __forceinline__ void fixed_tables(uint16_t *lens, HuffTab *hl, HuffTab *hd)
{
    const int l = lane_id();
    for (int s = l; s < 288; s += 64) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
    for (int s = l; s < 30; s += 64) lens[288 + s] = 5;
    __syncthreads();
    huff_build(hl, lens, 288, false);
    huff_build(hd, lens + 288, 30, true);
}

// ---- gz_find: grid nchunks x 64 ---------------------------------------------------------------
// start[c] = first bit offset in [c * kChunkBits, (c + 1) * kChunkBits) where a dynamic block header
// validates (chunk 0: bit 0), else -1.
__device__ __forceinline__ bool header_cheap(uint64_t lo64, uint32_t hi32)
{
    // BTYPE = 2, HLIT / HDIST in range, a complete code-length code; zlib's deflate trims trailing
    // zero code-length lengths (HCLEN = last nonzero + 1, at least 4) — a heuristic only: a start
    // it rejects is decoded through by the chunk before
    if (((lo64 >> 1) & 3) != 2) return false;
    const int nlit = (int)((lo64 >> 3) & 31), ndist = (int)((lo64 >> 8) & 31), ncl = (int)((lo64 >> 13) & 15) + 4;
    if (nlit > 29 || ndist > 29) return false;
    int left = 1 << 7, used = 0;
    uint32_t lastv = 0;
    for (int i = 0; i < ncl; i++) {
        const int at = 17 + 3 * i;
        const uint32_t v = at >= 64 ? (hi32 >> (at - 64)) & 7u
                         : at + 3 <= 64 ? (uint32_t)(lo64 >> at) & 7u
                                        : (uint32_t)(((lo64 >> at) | ((uint64_t)hi32 << (64 - at))) & 7u);
        if (v) { left -= 1 << (7 - v); used++; }
        lastv = v;
    }
    return left == 0 && used > 0 && (ncl == 4 || lastv != 0);
}

// grid nchunks x 64: the chunk's bytes staged in LDS; lane = byte, 8 bit offsets per lane
__global__ void __launch_bounds__(64) gz_find_kernel(const uint8_t *__restrict__ src, int64_t slen, int64_t *__restrict__ start)
{
    constexpr int kCB = (int)(kChunkBits / 8);        // chunk bytes
    __shared__ __attribute__((aligned(16))) uint32_t cb[kCB / 4 + 8];
    __shared__ __attribute__((aligned(16))) uint32_t stage[kInStage / 4];
    __shared__ HuffTab hl, hd;
    __shared__ uint16_t lens[320];
    const int c = blockIdx.x, l = lane_id();
    if (c == 0) { if (l == 0) start[0] = 0; return; }
    const int64_t B0 = (int64_t)c * kCB, hi = min(8 * (B0 + kCB), 8 * slen);
    for (int i = l; i < kCB / 4 + 8; i += 64) {        // bytes [B0, B0 + kCB + 32), zeros past the stream
        const int64_t o = B0 + 4 * i;
        uint32_t w = 0;
        if (o + 4 <= slen) w = rd32u(src + o);
        else for (int k = 0; k < 4; k++) if (o + k < slen) w |= (uint32_t)src[o + k] << (8 * k);
        cb[i] = w;
    }
    __syncthreads();
    BitIn in{src, slen, stage, -(int64_t)kInStage, 0, 0, 0};
    for (int by = 0; by < kCB; by += 64) {
        const int q = by + l;                          // this lane's byte (chunk-relative)
        const uint32_t w0 = cb[q >> 2], w1 = cb[(q >> 2) + 1], w2 = cb[(q >> 2) + 2], w3 = cb[(q >> 2) + 3];
        const uint32_t s8 = 8 * (q & 3);
        const uint32_t a0 = s8 ? (w0 >> s8) | (w1 << (32 - s8)) : w0;
        const uint32_t a1 = s8 ? (w1 >> s8) | (w2 << (32 - s8)) : w1;
        const uint32_t a2 = s8 ? (w2 >> s8) | (w3 << (32 - s8)) : w2;   // bytes q .. q + 11
        const uint64_t w = (uint64_t)a0 | ((uint64_t)a1 << 32);
        uint32_t mask = 0;
#pragma unroll
        for (int sh = 0; sh < 8; sh++) {
            const uint64_t lo64 = (w >> sh) | (sh ? ((uint64_t)a2 << (64 - sh)) : 0ull);
            const int64_t b = 8 * (B0 + q) + sh;
            if (b < hi && header_cheap(lo64, a2 >> sh)) mask |= 1u << sh;
        }
        unsigned long long m = ballot64(mask != 0);
        while (m) {                                    // full header decode, in bit order
            const int k = __builtin_ctzll(m);
            uint32_t mk = rdlane(mask, k);
            while (mk) {
                const int sh = __builtin_ctz(mk);
                mk &= mk - 1;
                const int64_t b = 8 * (B0 + by + k) + sh;
                in.start(b);
                in.bits(3);
                if (read_dynamic<false>(in, lens, &hl, &hd) == 0) {
                    if (l == 0) start[c] = b;
                    return;
                }
            }
            m &= m - 1;
        }
    }
    if (l == 0) start[c] = -1;
}

// ---- the chunk decoder -----------------------------------------------------------------------
// Decodes from bit `from` until a block ends at a bit offset equal to a later chunk start
// (kWrite = false: finds it and counts) or at `stop_bit` (kWrite = true).  Write mode keeps the
// output in an LDS ring of u16 values (bytes, or 256 + w for window byte w before the chunk) and
// flushes it to scratch[out0 ..] as u32 (markers as 256 + absolute source position).
struct ChunkOut {
    int64_t n;           // output bytes
    int64_t end_bit;     // bit offset after the last block decoded
    int end_chunk;       // chunk whose start it reached (nchunks: the final block), -1: error
    int final_block;
};

template <bool kWrite>
__device__ __forceinline__ ChunkOut decode_chunk(BitIn &in, int64_t from, const int64_t *starts, int c, int nchunks, int64_t stop_bit,
                                 uint16_t *lens, HuffTab *hl, HuffTab *hd, uint16_t *ring, uint32_t *scratch,
                                 int64_t out0, int64_t cap)
{
    const int l = lane_id();
    ChunkOut r{0, 0, -1, 0};
    in.start(from);
    int64_t pos = 0, flushed = 0;
    int j = c + 1;                                     // next candidate chunk start
    auto flush = [&](int64_t upto) {                   // ring [flushed, upto) -> scratch
        __syncthreads();
        for (int64_t i = flushed + l; i < upto; i += 64) {
            const uint32_t v = ring[i & (kRing - 1)];
            scratch[out0 + i] = v < 256u ? v : (uint32_t)(256 + (out0 - kRing + (int64_t)(v - 256u)));
        }
        flushed = upto;
    };
    for (;;) {
        const bool last = in.bits(1) != 0;
        const int type = (int)in.bits(2);
        if (type == 0) {                               // stored: byte-aligned LEN, NLEN, raw bytes
            const int drop = in.bn & 7;
            in.bb >>= drop;
            in.bn -= drop;
            const uint32_t len = in.bits(16), nlen = in.bits(16);
            const int64_t P = in.pos() >> 3;
            if ((len ^ 0xffffu) != nlen || P + (int64_t)len > in.slen) return r;
            if (kWrite) {
                if (pos + (int64_t)len > cap) return r;
                for (uint32_t o = 0; o < len; o += 1024) {  // 16 bytes per lane per step
                    const uint32_t q0 = o + 16 * l;
                    uint32_t w[4] = {0, 0, 0, 0};
                    if (q0 + 16 <= len) {
                        const uint8_t *sp = in.src + P + q0;
                        const uint8_t *sa = (const uint8_t *)((uintptr_t)sp & ~(uintptr_t)3);
                        const uint32_t sh = (uint32_t)((uintptr_t)sp & 3);
                        uint32_t a[5];
#pragma unroll
                        for (int t = 0; t < 5; t++) a[t] = (t < 4 || sh) ? ld4(sa + 4 * t) : 0u;
#pragma unroll
                        for (int t = 0; t < 4; t++) w[t] = __builtin_amdgcn_alignbyte(a[t + 1], a[t], sh);
                    } else {
                        for (uint32_t t = 0; t < 16 && q0 + t < len; t++) w[t >> 2] |= (uint32_t)in.src[P + q0 + t] << (8 * (t & 3));
                    }
#pragma unroll
                    for (int t = 0; t < 16; t++)
                        if (q0 + t < len) ring[(pos + q0 + t) & (kRing - 1)] = (uint16_t)((w[t >> 2] >> (8 * (t & 3))) & 0xffu);
                    const int64_t pw = pos + min(len, o + 1024);
                    if (pw - flushed >= kFlushAt) flush(flushed + kFlushAt);
                }
            }
            pos += len;
            in.start(8 * (P + (int64_t)len));
        } else if (type == 3) {
            return r;
        } else {
            if (type == 1) fixed_tables(lens, hl, hd);
            else if (read_dynamic(in, lens, hl, hd) != 0) return r;
            for (;;) {
                const int sym = in.decode(hl);
                if (sym < 0 || in.over()) return r;
                if (sym < 256) {
                    if (kWrite) {
                        if (pos >= cap) return r;
                        if (l == 0) ring[pos & (kRing - 1)] = (uint16_t)sym;
                    }
                    pos++;
                } else if (sym == 256) {
                    break;
                } else {
                    const int li = sym - 257;
                    if (li >= 29) return r;
                    const int len = kLenBase[li] + (int)in.bits(kLenExtra[li]);
                    const int ds = in.decode(hd);
                    if (ds < 0 || ds >= 30) return r;
                    const int dist = kDistBase[ds] + (int)in.bits(kDistExtra[ds]);
                    if (kWrite) {
                        if (pos + len > cap) return r;
                        if (c == 0 && dist > pos) return r;    // nothing before the first chunk
                        asm volatile("" ::: "memory");          // ring reads after the earlier writes
                        for (int o = 0; o < len; o += 64) {
                            const int i = o + l;
                            if (i < len) {
                                int q = i;                         // i mod dist without a division
                                while (q >= dist) q -= dist;
                                const int64_t sp = pos - dist + q;
                                const uint16_t v = sp >= 0 ? ring[sp & (kRing - 1)] : (uint16_t)(256 + (kRing + sp));
                                ring[(pos + i) & (kRing - 1)] = v;
                            }
                        }
                    } else if (c == 0 && dist > pos) {
                        return r;
                    }
                    pos += len;
                }
                if (kWrite && pos - flushed >= kFlushAt) flush(flushed + kFlushAt);
            }
        }
        const int64_t e = in.pos();
        if (kWrite) {
            if (last || e >= stop_bit) {
                flush(pos);
                r.n = pos; r.end_bit = e; r.end_chunk = 0; r.final_block = last;
                return r;
            }
        } else {
            if (last) {
                r.n = pos; r.end_bit = e; r.end_chunk = nchunks; r.final_block = 1;
                return r;
            }
            while (j < nchunks && (starts[j] < 0 || starts[j] < e)) j++;
            if (j < nchunks && starts[j] == e) {
                r.n = pos; r.end_bit = e; r.end_chunk = j;
                return r;
            }
        }
        if (e > 8 * in.slen + 64) return r;            // ran past the stream
    }
}

// grid nchunks x 64: info[c] = {output bytes, end bit, end chunk (-1 error), final}
__global__ void __launch_bounds__(64) gz_count_kernel(const uint8_t *__restrict__ src, int64_t slen,
                                                      const int64_t *__restrict__ starts, int nchunks,
                                                      int64_t *__restrict__ info)
{
    __shared__ __attribute__((aligned(16))) uint32_t stage[kInStage / 4];
    __shared__ HuffTab hl, hd;
    __shared__ uint16_t lens[320];
    const int c = blockIdx.x;
    const int64_t s = starts[c];
    int64_t *o = info + 4 * (size_t)c;
    if (s < 0) { if (lane_id() == 0) { o[0] = 0; o[1] = 0; o[2] = -1; o[3] = 0; } return; }
    BitIn in{src, slen, stage, -(int64_t)kInStage, 0, 0, 0};
    const ChunkOut r = decode_chunk<false>(in, s, starts, c, nchunks, 0, lens, &hl, &hd, nullptr, nullptr, 0, 0);
    if (lane_id() == 0) { o[0] = r.n; o[1] = r.end_bit; o[2] = r.end_chunk; o[3] = r.final_block; }
}

// grid nlist x 64: chain chunk k = list[k] -> scratch[out0[k] ..]; ok[k] = 1 on success
__global__ void __launch_bounds__(64) gz_write_kernel(const uint8_t *__restrict__ src, int64_t slen,
                                                      const int64_t *__restrict__ job, int njob,
                                                      uint32_t *__restrict__ scratch, int64_t cap, int *__restrict__ err)
{
    __shared__ __attribute__((aligned(16))) uint32_t stage[kInStage / 4];
    __shared__ HuffTab hl, hd;
    __shared__ uint16_t lens[320];
    __shared__ uint16_t ring[kRing];
    const int k = blockIdx.x;
    const int64_t *jb = job + 5 * (size_t)k;            // {start bit, stop bit, out0, n, chunk index}
    BitIn in{src, slen, stage, -(int64_t)kInStage, 0, 0, 0};
    const ChunkOut r = decode_chunk<true>(in, jb[0], nullptr, (int)jb[4], 0, jb[1], lens, &hl, &hd, ring, scratch, jb[2],
                                          cap - jb[2]);
    if (lane_id() == 0 && (r.end_chunk != 0 || r.n != jb[3] || r.end_bit != jb[1])) atomicOr(err, 1);
}

// one pointer-jumping pass: every marker takes what its source holds; *left counts markers seen
__global__ void __launch_bounds__(256) gz_resolve_kernel(uint32_t *__restrict__ s, int64_t n, unsigned int *__restrict__ left)
{
    unsigned int cnt = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint32_t v = s[i];
        if (v >= 256u) {
            const uint32_t w = s[v - 256u];
            s[i] = w;
            cnt += w >= 256u;
        }
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
    if (lane_id() == 0 && cnt) atomicAdd(left, cnt);
}

__global__ void __launch_bounds__(256) gz_pack_kernel(const uint32_t *__restrict__ s, int64_t n, uint8_t *__restrict__ dst)
{
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) dst[i] = (uint8_t)s[i];
}

// grid pieces x 64: crc[i] = CRC-32 of data[i * piece, min((i + 1) * piece, n)), piece = 64 KiB.
// Each lane takes 1 KiB (byte table in LDS); lane 0 folds the lane CRCs with the "append 1 KiB"
// operator (crc(A||B) = op(crc(A)) ^ crc(B)) and runs the tail bytes itself.
__global__ void __launch_bounds__(64) crc32_piece_kernel(const uint8_t *__restrict__ data, int64_t n, CrcOp op1k,
                                                         uint32_t *__restrict__ crc)
{
    __shared__ uint32_t tab[256];
    __shared__ uint32_t lc[64];
    const int l = lane_id();
    for (int t = l; t < 256; t += 64) {
        uint32_t c = (uint32_t)t;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        tab[t] = c;
    }
    __syncthreads();
    const int64_t a0 = (int64_t)blockIdx.x * 65536, pl = min((int64_t)65536, n - a0);
    const int nfull = (int)(pl >> 10);
    if (l < nfull) {
        const uint8_t *w = data + a0 + 1024 * l;       // any alignment (members follow each other)
        uint32_t r = 0xffffffffu;
        for (int i = 0; i < 256; i++) {
            // rd32u reads up to 3 bytes past its word: the last word by bytes (the buffer may end there)
            const uint32_t x = i < 255 ? rd32u(w + 4 * i)
                                       : (uint32_t)w[1020] | ((uint32_t)w[1021] << 8) | ((uint32_t)w[1022] << 16) |
                                             ((uint32_t)w[1023] << 24);
            r = tab[(r ^ x) & 0xff] ^ (r >> 8);
            r = tab[(r ^ (x >> 8)) & 0xff] ^ (r >> 8);
            r = tab[(r ^ (x >> 16)) & 0xff] ^ (r >> 8);
            r = tab[(r ^ (x >> 24)) & 0xff] ^ (r >> 8);
        }
        lc[l] = r ^ 0xffffffffu;
    }
    __syncthreads();
    if (l == 0) {
        uint32_t acc = 0;
        for (int i = 0; i < nfull; i++) {
            uint32_t s = 0, v = acc;
            for (int k = 0; v; v >>= 1, k++)
                if (v & 1) s ^= op1k.m[k];
            acc = i ? s ^ lc[i] : lc[0];
        }
        uint32_t r = acc ^ 0xffffffffu;                // continue the CRC over the tail bytes
        for (int64_t p = a0 + 1024 * (int64_t)nfull; p < a0 + pl; p++) r = tab[(r ^ data[p]) & 0xff] ^ (r >> 8);
        crc[blockIdx.x] = nfull || pl > 0 ? r ^ 0xffffffffu : 0u;
    }
}

int64_t inflate_chunks(int64_t slen) { return (8 * slen + kChunkBits - 1) / kChunkBits; }

hipError_t launch_inflate_find(const uint8_t *src, int64_t slen, int64_t *starts, int64_t *info, hipStream_t st)
{
    const int64_t n = inflate_chunks(slen);
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gz_find_kernel, dim3((unsigned)n), dim3(64), 0, st, src, slen, starts);
    hipLaunchKernelGGL(gz_count_kernel, dim3((unsigned)n), dim3(64), 0, st, src, slen, starts, (int)n, info);
    return hipGetLastError();
}

hipError_t launch_inflate_write(const uint8_t *src, int64_t slen, const int64_t *jobs, int njobs, uint32_t *scratch,
                                int64_t cap, int *err, hipStream_t st)
{
    if (njobs > 0)
        hipLaunchKernelGGL(gz_write_kernel, dim3((unsigned)njobs), dim3(64), 0, st, src, slen, jobs, njobs, scratch, cap, err);
    return hipGetLastError();
}

hipError_t launch_inflate_resolve(uint32_t *scratch, int64_t n, unsigned int *left, hipStream_t st)
{
    const unsigned g = (unsigned)std::min<int64_t>(8192, std::max<int64_t>(1, (n + 255) / 256));
    hipLaunchKernelGGL(gz_resolve_kernel, dim3(g), dim3(256), 0, st, scratch, n, left);
    return hipGetLastError();
}

hipError_t launch_inflate_pack(const uint32_t *scratch, int64_t n, uint8_t *dst, hipStream_t st)
{
    const unsigned g = (unsigned)std::min<int64_t>(8192, std::max<int64_t>(1, (n + 255) / 256));
    if (n > 0) hipLaunchKernelGGL(gz_pack_kernel, dim3(g), dim3(256), 0, st, scratch, n, dst);
    return hipGetLastError();
}

hipError_t launch_crc32_pieces(const uint8_t *data, int64_t n, const CrcOp &op1k, uint32_t *crc, hipStream_t st)
{
    const int64_t np = (n + 65535) / 65536;
    if (np > 0) hipLaunchKernelGGL(crc32_piece_kernel, dim3((unsigned)np), dim3(64), 0, st, data, n, op1k, crc);
    return hipGetLastError();
}

}  // namespace hdrf
