// corpus.hip — synthetic corpus generator (BASELINE configs 2 and 4; spec in DESIGN.md §Corpus).
// Block b is segs_per_block segments; segment s is filled with splitmix64 words keyed by
// roots[b*spb+s] (a segment chosen as a duplicate carries the root of an earlier block's
// segment, so its bytes repeat exactly).  Written 16 B per lane, coalesced.
// Mixed-entropy mode (config 4): each root also picks the segment's kind — random words, "text"
// (8-byte slots holding one of 512 seven-letter words + space) or "binary" (16-byte LE records
// {u32 index, u32 value < 200, u32 flags < 4, u32 0}); hdrf_amd/corpus.py mirrors it on the host.
#include "launchers.hpp"

namespace hdrf {

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t text_word(uint64_t k)
{
    const uint64_t m = mix64((k & 511) ^ 0x7E57ull);
    uint64_t w = 0;
#pragma unroll
    for (int j = 0; j < 7; j++) w |= (uint64_t)('a' + (uint32_t)((m >> (5 * j)) % 26)) << (8 * j);
    return w | ((uint64_t)' ' << 56);
}

__global__ void __launch_bounds__(256) corpus_kernel(uint8_t *__restrict__ dev, const uint32_t *__restrict__ roots,
                                                     int64_t nsegs, int64_t seg_bytes, uint64_t seed, int mixed)
{
    const int64_t pairs_per_seg = seg_bytes / 16;
    const int64_t total = nsegs * pairs_per_seg;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t sg = i / pairs_per_seg;
        const int64_t wi = (i - sg * pairs_per_seg) * 2;
        const uint64_t key = mix64(seed ^ mix64((uint64_t)roots[sg] + 1));
        uint64_t a = mix64(key + (uint64_t)wi), b = mix64(key + (uint64_t)wi + 1);
        if (mixed) {
            const uint32_t kind = (uint32_t)(mix64((uint64_t)roots[sg] ^ 0x5BD1E995ull) % 3);
            if (kind == 1) {
                a = text_word(a); b = text_word(b);
            } else if (kind == 2) {
                a = (uint64_t)(uint32_t)(wi >> 1) | ((a % 200) << 32);
                b = b % 4;
            }
        }
        ulonglong2 v; v.x = a; v.y = b;
        *reinterpret_cast<ulonglong2 *>(dev + sg * seg_bytes + wi * 8) = v;
    }
}

hipError_t launch_corpus(uint8_t *dev, const uint32_t *d_roots, int64_t nblocks, int64_t spb, int64_t seg_bytes,
                         uint64_t seed, int mixed, hipStream_t st)
{
    hipLaunchKernelGGL(corpus_kernel, dim3(256 * 16), dim3(256), 0, st, dev, d_roots, nblocks * spb, seg_bytes, seed,
                       mixed);
    return hipGetLastError();
}

}  // namespace hdrf
