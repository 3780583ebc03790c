// sha_peak.hip — compute ceiling of the SHA-1 compression as written in hdrf_amd/csrc/sha.hip:
// one chain per lane, message words in registers (no memory traffic), 80 rounds per call
// (Ch/Maj as single v_bitop3, as in the kernel).  Build: hipcc -O3 --offload-arch=gfx950.
// Prints compressions/s and the equivalent GB/s of hashed input for 4 and 8 waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

__device__ __forceinline__ void sha1_compress(uint32_t st[5], uint32_t w[16])
{
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
#pragma unroll
    for (int i = 0; i < 80; i++) {
        if (i >= 16) w[i & 15] = rotl(xor3(w[(i - 3) & 15], w[(i - 8) & 15], w[(i - 14) & 15]) ^ w[i & 15], 1);
        uint32_t f, k;
        if (i < 20)      { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xCA); k = 0x5A827999u; }
        else if (i < 40) { f = xor3(b, c, d);     k = 0x6ED9EBA1u; }
        else if (i < 60) { f = __builtin_amdgcn_bitop3_b32(b, c, d, 0xE8); k = 0x8F1BBCDCu; }
        else             { f = xor3(b, c, d);     k = 0xCA62C1D6u; }
        const uint32_t t = rotl(a, 5) + f + e + k + w[i & 15];
        e = d; d = c; c = rotl(b, 30); b = a; a = t;
    }
    st[0] += a; st[1] += b; st[2] += c; st[3] += d; st[4] += e;
}

template <int CH>
__global__ void __launch_bounds__(256) k(uint32_t *out, int iters)
{
    uint32_t st[CH][5], w[CH][16];
#pragma unroll
    for (int c = 0; c < CH; c++) {
#pragma unroll
        for (int i = 0; i < 5; i++) st[c][i] = threadIdx.x * 31 + i + c;
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int c = 0; c < CH; c++) {
#pragma unroll
            for (int i = 0; i < 16; i++) w[c][i] = st[c][i % 5] + i + it;
            sha1_compress(st[c], w[c]);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) x ^= st[c][0] ^ st[c][4];
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int CH>
static void run(int waves_per_simd, uint32_t *d)
{
    const int blocks = 256 * waves_per_simd, iters = 256;    // 256-thread WGs: 4 waves each, 1 per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(256), 0, 0, d, 4);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(256), 0, 0, d, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double comps = (double)blocks * 256 * iters * CH;
    printf("chains/lane %d  waves/SIMD %d: %8.3f ms  %.2f G compressions/s  = %.0f GB/s hashed\n", CH, waves_per_simd, ms,
           comps / ms / 1e6, comps * 64 / ms / 1e6);
}

int main()
{
    uint32_t *d;
    hipMalloc(&d, 256 * 8 * 256 * 4);
    run<1>(4, d); run<1>(8, d); run<2>(4, d); run<2>(2, d);
    hipFree(d);
    return 0;
}
