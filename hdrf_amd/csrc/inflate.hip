// inflate.hip — GzipCodec read side (DataNode.compressor 5) on gfx950: RFC 1951 inflate of a gzip
// member's deflate stream, plus the CRC-32 of the output.
//
// Reference: DN/DataConstructor.java:194-218 — a compressor-5 block file is read back through
// GzipCodec.createInputStream (Hadoop's DecompressorStream over zlib inflate, hadoop-common 3.1.0);
// tests check the output byte for byte against Python's zlib.decompress of the same file.
//
// A deflate stream is one sequential bit stream (each block's start is known only once the one
// before it is decoded), so one wave decodes one member, with everything it touches per symbol in
// LDS: the compressed input staged 4 KiB at a time, the Huffman tables (10-bit direct lookup +
// canonical slow path for longer codes), and a 64 KiB output ring holding the 32 KiB window.
// Literals are single LDS stores; a match is copied by the whole wave (lane i writes byte i of
// each 64-B step from ring[pos - dist + (i mod dist)], which is exact for overlapping copies);
// the ring is flushed to HBM in 16 KiB pieces of 16-B stores.  The CRC-32 runs afterwards, one
// thread per 64 KiB piece (byte table in LDS); the host combines the piece CRCs
// (crc32_combine, zlib's published GF(2) method).
#include "launchers.hpp"

namespace hdrf {

constexpr int kInRing = 4096;                // staged input bytes
constexpr int kOutRing = 65536;              // output ring (>= 32 KiB window + unflushed)
constexpr int kFlushStep = 16384;
constexpr int kFastBits = 10;

struct HuffTab {
    uint16_t fast[1 << kFastBits];            // (len << 9) | symbol for codes <= 10 bits, 0 = slow path
    uint16_t count[16];                       // codes per length
    uint16_t sym[320];                        // symbols in canonical order
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

typedef __attribute__((address_space(3))) volatile uint8_t lds_vu8;

// Build the decode tables from n code lengths (wave-cooperative).  Returns false on an
// over-subscribed set (an incomplete set is legal for the distance codes).
__device__ bool huff_build(HuffTab *t, const uint16_t *len, int n)
{
    const int l = lane_id();
    for (int i = l; i < (1 << kFastBits); i += 64) t->fast[i] = 0;
    if (l < 16) t->count[l] = 0;
    __syncthreads();
    if (l == 0) {
        for (int s = 0; s < n; s++) t->count[len[s]]++;
        t->count[0] = 0;
    }
    __syncthreads();
    uint16_t offs[16];
    int left = 1;
    bool ok = true;
    for (int b = 1; b < 16; b++) {
        left = (left << 1) - t->count[b];
        if (left < 0) ok = false;
    }
    offs[1] = 0;
    for (int b = 1; b < 15; b++) offs[b + 1] = offs[b] + t->count[b];
    if (l == 0)
        for (int s = 0; s < n; s++)
            if (len[s]) t->sym[offs[len[s]]++] = (uint16_t)s;
    __syncthreads();
    // direct table: canonical code of each symbol (codes of one length are consecutive), bit-reversed
    if (l == 0) {
        int code = 0, k = 0;
        for (int b = 1; b <= kFastBits; b++) {
            for (int c = 0; c < t->count[b]; c++, k++, code++) {
                int r = 0;
                for (int i = 0; i < b; i++) r |= ((code >> i) & 1) << (b - 1 - i);
                for (int f = r; f < (1 << kFastBits); f += 1 << b) t->fast[f] = (uint16_t)((b << 9) | t->sym[k]);
            }
            code <<= 1;
        }
    }
    __syncthreads();
    return ok;
}

// grid 1 x 64: inflate one raw deflate stream src[0, slen) into dst[0, cap).
// res[0] = output length (or < 0: error), res[1] = input bytes consumed (byte-aligned end)
__global__ void __launch_bounds__(64) gz_inflate_kernel(const uint8_t *__restrict__ src, int64_t slen,
                                                        uint8_t *__restrict__ dst, int64_t cap,
                                                        int64_t *__restrict__ res)
{
    __shared__ __attribute__((aligned(16))) uint8_t ring[kOutRing];
    __shared__ __attribute__((aligned(16))) uint8_t inb[kInRing + 16];
    __shared__ HuffTab hl, hd;
    __shared__ uint16_t lens[320];
    const int l = lane_id();
    lds_vu8 *vring = (lds_vu8 *)ring;
    // ---- bit reader over the staged input ---------------------------------------------------
    int64_t ibase = -(int64_t)kInRing;        // input staged: src[ibase, ibase + kInRing)
    int64_t ip = 0;                           // next byte to take into the bit buffer
    uint64_t bb = 0;
    int bn = 0;
    int err = 0;
    auto stage = [&](int64_t at) {            // stage src[at & ~15, +4096) (zero past slen)
        ibase = at & ~(int64_t)15;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int64_t o = ibase + 16 * (l + 64 * k);
            uint4 v;
            if (o + 16 <= slen) v = ld16(src + o);
            else {
                uint32_t w[4] = {0, 0, 0, 0};
                for (int i = 0; i < 16; i++)
                    if (o + i < slen) w[i >> 2] |= (uint32_t)src[o + i] << (8 * (i & 3));
                v = make_uint4(w[0], w[1], w[2], w[3]);
            }
            *(uint4 *)(inb + 16 * (l + 64 * k)) = v;
        }
        __syncthreads();
    };
    auto byte_at = [&](int64_t p) -> uint32_t {
        if (p < ibase || p >= ibase + kInRing) stage(p);
        return inb[p - ibase];
    };
    auto refill = [&]() {
        while (bn <= 56) {
            if (ip >= slen + 8) { err = -1; return; }            // ran past the stream
            bb |= (uint64_t)byte_at(ip) << bn;
            ip++;
            bn += 8;
        }
    };
    auto bits = [&](int n) -> uint32_t {      // n <= 32
        if (bn < n) refill();
        const uint32_t v = (uint32_t)(bb & ((n == 32) ? 0xffffffffull : ((1ull << n) - 1)));
        bb >>= n;
        bn -= n;
        return v;
    };
    auto decode = [&](const HuffTab *t) -> int {
        if (bn < 15) refill();
        const uint32_t e = t->fast[bb & ((1u << kFastBits) - 1)];
        if (e) {
            const int n = e >> 9;
            bb >>= n;
            bn -= n;
            return e & 511;
        }
        // canonical decode, one bit at a time (codes longer than 10 bits)
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
    };
    int64_t pos = 0, flushed = 0;
    auto flush = [&](int64_t upto) {          // ring bytes [flushed, upto) -> dst (upto - flushed <= 16 KiB)
        __syncthreads();
        const int64_t n = upto - flushed;
        const int off = (int)(flushed & (kOutRing - 1));        // multiple of 16 except the final piece
        const int nw = ((uintptr_t)dst & 15) ? 0 : (int)(n >> 4);   // 16-B stores need an aligned dst
        for (int w = l; w < nw; w += 64) {
            const uint4 v = *(const uint4 *)(ring + off + 16 * w);
            st16(dst + flushed + 16 * w, v);
        }
        for (int64_t i = 16 * (int64_t)nw + l; i < n; i += 64) dst[flushed + i] = ring[(off + i) & (kOutRing - 1)];
        flushed = upto;
    };
    bool last = false;
    while (!last && !err) {
        last = bits(1);
        const int type = (int)bits(2);
        if (type == 0) {                       // stored: byte-align, LEN, NLEN, LEN raw bytes
            const int drop = bn & 7;
            bb >>= drop;
            bn -= drop;
            ip -= bn >> 3;                     // hand the buffered bytes back to the byte reader
            bb = 0;
            bn = 0;
            const uint32_t len = byte_at(ip) | (byte_at(ip + 1) << 8);
            const uint32_t nlen = byte_at(ip + 2) | (byte_at(ip + 3) << 8);
            ip += 4;
            if ((len ^ 0xffffu) != nlen || ip + len > slen || pos + len > cap) { err = -2; break; }
            // 4 KiB steps (16 B per lane), flushing between steps so the ring never overruns
            for (uint32_t o = 0; o < len; o += 1024) {
                const int64_t q = ip + o + 16 * l;
                if (o + 16 * l < len) {
                    const uint32_t nb = min(16u, len - (o + 16 * l));
                    for (uint32_t j = 0; j < nb; j++)
                        vring[(pos + o + 16 * l + j) & (kOutRing - 1)] = src[q + j];
                }
                if (((o + 1024) & 4095) == 0 || o + 1024 >= len) {
                    const int64_t at = pos + min(len, o + 1024);
                    while (at - flushed >= kFlushStep) flush(flushed + kFlushStep);
                }
            }
            ip += len;
            pos += len;
            continue;
        }
        if (type == 3) { err = -3; break; }
        // ---- code tables ------------------------------------------------------------------------
        int nlit = 288, ndist = 30;
        if (type == 1) {                       // fixed codes
            for (int s = l; s < 288; s += 64) lens[s] = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8;
            for (int s = l; s < 30; s += 64) lens[288 + s] = 5;
            __syncthreads();
        } else {                               // dynamic codes
            nlit = (int)bits(5) + 257;
            ndist = (int)bits(5) + 1;
            const int ncl = (int)bits(4) + 4;
            if (nlit > 286 || ndist > 30) { err = -4; break; }
            for (int s = l; s < 19; s += 64) lens[s] = 0;
            __syncthreads();
            for (int i = 0; i < ncl; i++) {
                const uint32_t v = bits(3);
                if (l == 0) lens[kClOrder[i]] = (uint16_t)v;
            }
            __syncthreads();
            if (!huff_build(&hl, lens, 19)) { err = -5; break; }
            int i = 0;
            uint16_t prev = 0;
            while (i < nlit + ndist) {
                const int sym = decode(&hl);
                if (sym < 0) { err = -6; break; }
                int rep = 1;
                uint16_t v = (uint16_t)sym;
                if (sym == 16) { if (i == 0) { err = -7; break; } v = prev; rep = 3 + (int)bits(2); }
                else if (sym == 17) { v = 0; rep = 3 + (int)bits(3); }
                else if (sym == 18) { v = 0; rep = 11 + (int)bits(7); }
                if (i + rep > nlit + ndist) { err = -8; break; }
                __syncthreads();
                for (int k = l; k < rep; k += 64) lens[i + k] = v;
                __syncthreads();
                i += rep;
                prev = v;
            }
            if (err) break;
            if (lens[256] == 0) { err = -9; break; }
            // the distance lengths follow the literal/length ones: move them to lens[288..]
            __syncthreads();
            uint16_t dv = l < ndist ? lens[nlit + l] : 0;
            __syncthreads();
            if (l < 30) lens[288 + l] = l < ndist ? dv : 0;
            for (int s = nlit + l; s < 288; s += 64) lens[s] = 0;
            __syncthreads();
        }
        if (!huff_build(&hl, lens, 288)) { err = -10; break; }
        {
            bool ok = huff_build(&hd, lens + 288, 30);
            (void)ok;                          // an incomplete distance set is legal
        }
        // ---- symbols -------------------------------------------------------------------------------
        for (;;) {
            const int sym = decode(&hl);
            if (sym < 0) { err = -11; break; }
            if (sym < 256) {
                if (pos >= cap) { err = -12; break; }
                if (l == 0) vring[pos & (kOutRing - 1)] = (uint8_t)sym;
                pos++;
            } else if (sym == 256) {
                break;
            } else {
                const int li = sym - 257;
                if (li >= 29) { err = -13; break; }
                const int len = kLenBase[li] + (int)bits(kLenExtra[li]);
                const int ds = decode(&hd);
                if (ds < 0 || ds >= 30) { err = -14; break; }
                const int dist = kDistBase[ds] + (int)bits(kDistExtra[ds]);
                if (dist > pos) { err = -15; break; }
                if (pos + len > cap) { err = -12; break; }
                for (int o = 0; o < len; o += 64) {
                    const int i = o + l;
                    if (i < len) {
                        const int q = dist >= len ? i : i % dist;
                        const uint8_t b = vring[(pos - dist + q) & (kOutRing - 1)];
                        vring[(pos + i) & (kOutRing - 1)] = b;
                    }
                }
                pos += len;
            }
            if (pos - flushed >= kFlushStep) flush(flushed + kFlushStep);
        }
    }
    if (!err) flush(pos);
    if (l == 0) {
        res[0] = err ? (int64_t)err : pos;
        res[1] = ip - (bn >> 3);              // bytes consumed (the unread whole bytes go back)
    }
}

// grid ceil(pieces / 256) x 256: crc[i] = CRC-32 of dst[i * piece, min((i + 1) * piece, n))
__global__ void __launch_bounds__(256) crc32_piece_kernel(const uint8_t *__restrict__ data, int64_t n, int64_t piece,
                                                          uint32_t *__restrict__ crc)
{
    __shared__ uint32_t tab[256];
    const int t = threadIdx.x;
    uint32_t c = (uint32_t)t;
    for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    tab[t] = c;
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * 256 + t;
    const int64_t a = i * piece, b = min(n, a + piece);
    if (a >= n) return;
    uint32_t r = 0xffffffffu;
    int64_t p = a;
    for (; p + 4 <= b && (p & 3); p++) r = tab[(r ^ data[p]) & 0xff] ^ (r >> 8);
    for (; p + 4 <= b; p += 4) {
        const uint32_t w = *(const uint32_t *)(data + p);
        r = tab[(r ^ w) & 0xff] ^ (r >> 8);
        r = tab[(r ^ (w >> 8)) & 0xff] ^ (r >> 8);
        r = tab[(r ^ (w >> 16)) & 0xff] ^ (r >> 8);
        r = tab[(r ^ (w >> 24)) & 0xff] ^ (r >> 8);
    }
    for (; p < b; p++) r = tab[(r ^ data[p]) & 0xff] ^ (r >> 8);
    crc[i] = r ^ 0xffffffffu;
}

hipError_t launch_inflate(const uint8_t *src, int64_t slen, uint8_t *dst, int64_t cap, int64_t *res, hipStream_t st)
{
    hipLaunchKernelGGL(gz_inflate_kernel, dim3(1), dim3(64), 0, st, src, slen, dst, cap, res);
    return hipGetLastError();
}

hipError_t launch_crc32_pieces(const uint8_t *data, int64_t n, int64_t piece, uint32_t *crc, hipStream_t st)
{
    const int64_t np = (n + piece - 1) / piece;
    if (np > 0) hipLaunchKernelGGL(crc32_piece_kernel, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, st, data, n, piece, crc);
    return hipGetLastError();
}

}  // namespace hdrf
