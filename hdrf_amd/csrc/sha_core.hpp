// sha_core.hpp — SHA-1 / SHA-224 compression, FIPS 180-4 padding and the per-lane window loads
// shared by the fingerprint kernels (sha.hip) and the fused chunk + fingerprint pass (lanehash.hip).
// Reference: DN/utilities.java:98-137 (nayuki native compress + FIPS 180-4 padding).
#pragma once
#include "launchers.hpp"

namespace hdrf {

typedef uint32_t u32x4a __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
// one v_bitop3_b32 each (truth tables over src0 = 0xF0, src1 = 0xCC, src2 = 0xAA)
__device__ __forceinline__ uint32_t ch(uint32_t x, uint32_t y, uint32_t z) { return __builtin_amdgcn_bitop3_b32(x, y, z, 0xCA); }
__device__ __forceinline__ uint32_t maj(uint32_t x, uint32_t y, uint32_t z) { return __builtin_amdgcn_bitop3_b32(x, y, z, 0xE8); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c)
{
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);   // symmetric truth table: a ^ b ^ c
}

__device__ __forceinline__ void sha1_compress(uint32_t st[5], uint32_t w[16])
{
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
#pragma unroll
    for (int i = 0; i < 80; i++) {
        if (i >= 16) w[i & 15] = rotl(xor3(w[(i - 3) & 15], w[(i - 8) & 15], w[(i - 14) & 15]) ^ w[i & 15], 1);
        uint32_t f, k;
        if (i < 20)      { f = ch(b, c, d);       k = 0x5A827999u; }
        else if (i < 40) { f = xor3(b, c, d);     k = 0x6ED9EBA1u; }
        else if (i < 60) { f = maj(b, c, d);      k = 0x8F1BBCDCu; }
        else             { f = xor3(b, c, d);     k = 0xCA62C1D6u; }
        const uint32_t t = rotl(a, 5) + f + e + k + w[i & 15];
        e = d; d = c; c = rotl(b, 30); b = a; a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

// (sha.hip defines the table with external linkage, as before the split; another translation unit
// including this header defines HDRF_SHA_K256_LINKAGE static, or the host shadows would collide)
#ifndef HDRF_SHA_K256_LINKAGE
#define HDRF_SHA_K256_LINKAGE
#endif
HDRF_SHA_K256_LINKAGE __constant__ uint32_t kK256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ void sha256_compress(uint32_t st[8], uint32_t w[16])
{
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
#pragma unroll
    for (int i = 0; i < 64; i++) {
        if (i >= 16) {
            const uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
            const uint32_t s0 = xor3(rotr(w15, 7), rotr(w15, 18), w15 >> 3);
            const uint32_t s1 = xor3(rotr(w2, 17), rotr(w2, 19), w2 >> 10);
            w[i & 15] = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
        }
        const uint32_t S1 = xor3(rotr(e, 6), rotr(e, 11), rotr(e, 25));
        const uint32_t t1 = h + S1 + ch(e, f, g) + kK256[i] + w[i & 15];
        const uint32_t S0 = xor3(rotr(a, 2), rotr(a, 13), rotr(a, 22));
        const uint32_t t2 = S0 + maj(a, b, c);
        h = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

template <int HW>
__device__ __forceinline__ void set_iv(uint32_t st[8])
{
    if (HW == 5) {
        st[0] = 0x67452301u; st[1] = 0xEFCDAB89u; st[2] = 0x98BADCFEu; st[3] = 0x10325476u; st[4] = 0xC3D2E1F0u;
        st[5] = st[6] = st[7] = 0u;
    } else {
        st[0] = 0xc1059ed8u; st[1] = 0x367cd507u; st[2] = 0x3070dd17u; st[3] = 0xf70e5939u;
        st[4] = 0xffc00b31u; st[5] = 0x68581511u; st[6] = 0x64f98fa7u; st[7] = 0xbefa4fa4u;
    }
}

// FIPS 180-4 padding of block j of a len-byte message, in place on its big-endian words: the
// message bytes [64 j, len) kept, 0x80 right after them, zeros, and the bit length in words 14-15
// of the last block (j == nb - 1).  A block the message fills (64 j + 64 <= len) is left unchanged,
// so the whole wave may run it.  e < 0: the length-only block after a tail of >= 56 bytes.
__device__ __forceinline__ void pad_block(uint32_t m[16], uint32_t len, uint32_t j, uint32_t nb)
{
    const int e = (int)len - 64 * (int)j;
    const int wt = e >> 2;                               // the word that takes the 0x80 byte
    const uint32_t rb = (uint32_t)e & 3u;
    const uint32_t hm = rb ? (0xffffffffu << (32 - 8 * rb)) : 0u;
    const uint32_t tb = e >= 0 ? (0x80000000u >> (8 * rb)) : 0u;
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = i < wt ? m[i] : (i == wt ? ((m[i] & hm) | tb) : 0u);
    if (j == nb - 1) {
        m[14] = len >> 29;
        m[15] = len << 3;
    }
}

// One iteration of a lane's compression chain (DN/utilities.java:98-137 over one chunk): blocks bi
// and, when `two`, bi + 1 from one 132-B window, so each 128-B line of the chunk is fetched once per
// pair (one block per iteration read every line twice, far apart in time: L2 misses 2.3x the
// algorithmic bytes).  The pairing is aligned so that the block T holding the message end is the
// SECOND of a pair (a chunk whose T is even starts with one single block): only slot 1 pads in
// steady state, and slot 0 only for T == 0 (a chunk under 64 B) or the length-only block T + 1.
// The padding is wave-uniform (ballot) because nearly every iteration has some lane at its tail;
// for the lanes not at their tail it changes nothing.
// The 33 dwords (132 B) of a window at pos (4-aligned down); `two`: both blocks of a pair.  Near
// the end of the readable bytes the guarded path reads past-the-end bytes as 0 (padding hides them).
__device__ __forceinline__ void load_win(const uint8_t *base, uint64_t readable, uint32_t pos, bool two, uint32_t d[33])
{
    const uint32_t apos = pos & ~3u;
    if ((uint64_t)apos + 132u <= readable) {          // all but a block's last chunk
        const HDRF_GLOBAL uint32_t *p = gptr<uint32_t>(base + apos);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            u32x4a v = *(const HDRF_GLOBAL u32x4a *)(p + 4 * q);
            d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
        }
        d[16] = p[16];
        if (two) {
#pragma unroll
            for (int q = 0; q < 4; q++) {
                u32x4a v = *(const HDRF_GLOBAL u32x4a *)(p + 17 + 4 * q);
                d[17 + 4 * q] = v.x; d[18 + 4 * q] = v.y; d[19 + 4 * q] = v.z; d[20 + 4 * q] = v.w;
            }
        }
    } else {
#pragma unroll
        for (int q = 0; q < 33; q++) d[q] = load4_guard(base, (int64_t)apos + 4 * q, (int64_t)readable);
    }
}

}  // namespace hdrf
