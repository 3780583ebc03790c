// bytes.hpp — byte-granular device helpers shared by the codec kernels (lz4.hip, snappy.hip).
#pragma once
#include "launchers.hpp"

namespace hdrf {

__device__ __forceinline__ uint32_t rd32u(const uint8_t *p)
{
    const uintptr_t a = (uintptr_t)p;
    const HDRF_GLOBAL uint32_t *q = gptr<uint32_t>((const void *)(a & ~(uintptr_t)3));
    return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}
// the 4 bytes at base + off, for a wave-uniform base: one global_load_dword with the base in SGPRs
// and a 32-bit lane offset (the amdhsa target runs with unaligned global access enabled, so the
// unaligned dword is a single load, against rd32u's aligned pair, 64-bit address and alignbyte)
__device__ __forceinline__ uint32_t ld32u(const uint8_t *base, uint32_t off)
{
    typedef uint32_t __attribute__((aligned(1))) u32u;
    return *gptr<u32u>((const void *)(base + off));
}
__device__ __forceinline__ uint32_t rd8(const uint8_t *p) { return *(const HDRF_GLOBAL uint8_t *)p; }
__device__ __forceinline__ void wr8(uint8_t *p, uint32_t v) { *(HDRF_GLOBAL uint8_t *)p = (uint8_t)v; }

// wave-cooperative copy of n bytes (arbitrary alignments; 16-B aligned destination words)
__device__ inline void wave_copy(uint8_t *dst, const uint8_t *src, int n)
{
    const int l = lane_id();
    int head = (int)((16 - ((uintptr_t)dst & 15)) & 15);
    if (head > n) head = n;
    if (l < head) wr8(dst + l, rd8(src + l));
    uint8_t *d = dst + head;
    const uint8_t *sp = src + head;
    const int n16 = (n - head) >> 4;
    const int sh = (int)((uintptr_t)sp & 15);
    const uint8_t *sa = sp - sh;
    int i = l;
    for (; i + 192 < n16; i += 256) {                 // four 16-B words per lane in flight
        const uint4 v0 = load16_shift(sa + 16 * (size_t)i, sh);
        const uint4 v1 = load16_shift(sa + 16 * (size_t)(i + 64), sh);
        const uint4 v2 = load16_shift(sa + 16 * (size_t)(i + 128), sh);
        const uint4 v3 = load16_shift(sa + 16 * (size_t)(i + 192), sh);
        st16(d + 16 * (size_t)i, v0);
        st16(d + 16 * (size_t)(i + 64), v1);
        st16(d + 16 * (size_t)(i + 128), v2);
        st16(d + 16 * (size_t)(i + 192), v3);
    }
    for (; i < n16; i += 64) st16(d + 16 * (size_t)i, load16_shift(sa + 16 * (size_t)i, sh));
    const int tb = head + 16 * n16;
    for (int k = tb + l; k < n; k += 64) wr8(dst + k, rd8(src + k));
}

__device__ __forceinline__ void put_be32(uint8_t *p, uint32_t v)
{
    wr8(p, v >> 24); wr8(p + 1, v >> 16); wr8(p + 2, v >> 8); wr8(p + 3, v);
}

}  // namespace hdrf
