// mall_probe.hip — Infinity-Cache (MALL) reuse probe for the batch-schedule design.
// Questions: does a second streaming read of an X-MiB buffer run faster than the first (served
// on-die), up to which X; do nontemporal loads allocate in the Infinity Cache; how much other
// traffic between two reads of the same bytes still leaves them resident.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mall_probe.hip -o tools/_build/mall_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void rd(const u32x4 *__restrict__ p, uint64_t n16, uint32_t *out)
{
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride * 4) {
        u32x4 v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint64_t j = i + k * stride;
            if (j < n16) v[k] = NT ? __builtin_nontemporal_load(p + j) : p[j];
            else v[k] = u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int k = 0; k < 4; k++) acc ^= v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ void fill(u32x4 *p, uint64_t n16, uint32_t s)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * 256)
        p[i] = u32x4{(uint32_t)i ^ s, (uint32_t)(i >> 7) * 3u, s, (uint32_t)i * 2654435761u};
}

static hipEvent_t e0, e1;
static uint32_t *d_out;

static float timed(const void *p, uint64_t bytes, bool nt)
{
    const int grid = 256 * 16;
    hipEventRecord(e0);
    if (nt) rd<true><<<grid, 256>>>((const u32x4 *)p, bytes / 16, d_out);
    else rd<false><<<grid, 256>>>((const u32x4 *)p, bytes / 16, d_out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main()
{
    const uint64_t MiB = 1ull << 20, FL = 2048 * MiB, BIG = 512 * MiB;
    uint8_t *F, *A, *B;
    CK(hipMalloc(&F, FL));
    CK(hipMalloc(&A, BIG));
    CK(hipMalloc(&B, BIG));
    CK(hipMalloc(&d_out, 65536 * 4));
    fill<<<4096, 256>>>((u32x4 *)F, FL / 16, 1);
    fill<<<4096, 256>>>((u32x4 *)A, BIG / 16, 2);
    fill<<<4096, 256>>>((u32x4 *)B, BIG / 16, 3);
    CK(hipDeviceSynchronize());
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto gbs = [](uint64_t b, float ms) { return b / (ms * 1e-3) / 1e9; };
    timed(F, FL, false);
    printf("flush buffer %.0f GB/s\n", gbs(FL, timed(F, FL, false)));
    // 1. re-read of X MiB right after the first read
    const int xs[] = {16, 32, 64, 128, 160, 192, 224, 256, 320, 512};
    for (int nt = 0; nt < 2; nt++)
        for (int x : xs) {
            const uint64_t b = x * MiB;
            float t1 = 0, t2 = 0;
            for (int r = 0; r < 3; r++) {
                timed(F, FL, false);                   // evict
                t1 += timed(A, b, nt);
                t2 += timed(A, b, false);
            }
            printf("reread  X=%4d MiB first=%s  first %7.0f GB/s  second %7.0f GB/s\n", x, nt ? "nt " : "def",
                   gbs(b, t1 / 3), gbs(b, t2 / 3));
        }
    // 2. reuse distance: read A (X), then Y MiB of other bytes, then A again
    const int ax[] = {64, 128};
    const int ys[] = {0, 32, 64, 128, 192, 256};
    for (int x : ax)
        for (int y : ys) {
            const uint64_t b = x * MiB;
            float t2 = 0;
            for (int r = 0; r < 3; r++) {
                timed(F, FL, false);
                timed(A, b, false);
                if (y) timed(B, y * MiB, false);
                t2 += timed(A, b, false);
            }
            printf("distance X=%4d MiB then %4d MiB other: reread %7.0f GB/s\n", x, y, gbs(b, t2 / 3));
        }
    printf("done\n");
    return 0;
}
