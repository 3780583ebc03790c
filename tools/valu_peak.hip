// valu_peak.hip — measured integer VALU issue rate on gfx950 for the SHA instruction mix
// (v_alignbit_b32, v_add3_u32, v_bitop3_b32, v_add_u32).  8 independent chains per lane,
// 32 waves per CU, timed with hipEvents.  Prints wave-instructions per cycle per SIMD and the
// chip-wide lane-op rate used as the SHA kernels' roofline denominator.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint32_t s, int iters)
{
    uint32_t a[8];
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = threadIdx.x * 7 + i + s;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int r = 0; r < 16; r++) {
#pragma unroll
            for (int i = 0; i < 8; i++) {
                if (OP == 0) a[i] = __builtin_amdgcn_alignbit(a[i], a[(i + 1) & 7], 5);
                else if (OP == 1) a[i] = a[i] + a[(i + 1) & 7] + a[(i + 3) & 7];
                else if (OP == 2) a[i] = __builtin_amdgcn_bitop3_b32(a[i], a[(i + 1) & 7], a[(i + 2) & 7], 0x96);
                else a[i] = a[i] + a[(i + 5) & 7];
            }
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) x ^= a[i];
    out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int OP>
static void run(const char *name, uint32_t *d)
{
    const int blocks = 256 * 8, iters = 4096;
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 1u, 16);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, d, 2u, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double winst = (double)blocks * 4 * iters * 16 * 8;       // wave-instructions
    const double lane_ops = winst * 64;
    printf("%-10s %8.3f ms  %.2f Tlane-op/s  %.3f wave-instr/ns\n", name, ms, lane_ops / ms / 1e9, winst / ms / 1e6);
}

int main()
{
    uint32_t *d;
    hipMalloc(&d, 256 * 8 * 256 * 4);
    run<0>("alignbit", d);
    run<1>("add3", d);
    run<2>("bitop3", d);
    run<3>("add_u32", d);
    hipFree(d);
    return 0;
}
