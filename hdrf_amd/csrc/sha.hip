// sha.hip — per-chunk SHA-1 / SHA-224 fingerprints on gfx950 (integer VALU, no MFMA).
//
// Reference: threadedHasher.run, DN/DataDeduplicator.java:578-641 hashes chunk k =
// [off[k-1], off[k]) with utilities.sha1hash (hasher==0) or sha224hash (hasher==1),
// DN/utilities.java:98-137 (nayuki native compress + FIPS 180-4 padding).
//
// One kernel: sha_chunk — a lane owns one chunk's whole compression chain, FIPS
// 180-4 padding and digest included; a lane that finishes its chunk immediately takes the next one
// from the wave's register pool of reserved chunks (ballot + mbcnt + ds_bpermute), so lanes do not
// idle while the wave's longest chunk finishes.
// Each 64-B block is fetched as 17 dword-aligned dwords (4 x dwordx4 + 1) and realigned +
// byte-swapped with one v_perm_b32 per word.  Rotations are v_alignbit_b32, 3-way xor is
// v_bitop3_b32 (gfx950), and so are Ch and Maj (one v_bitop3 each: 618 VALU per SHA-1 block).
// Lanes hash two consecutive blocks per iteration from one 132-B window (4 + 4 dwordx4 + 1 dword).
// A lane with one block left idles through the second compression.
// Measured against tools/sha_peak.hip (the same compression on register-resident data, no memory):
// a software-pipelined prefetch variant and a two-chains-per-lane variant were both slower, and so
// were nontemporal loads for the part of each window read for the last time (r03: 800 vs 980 GB/s,
// more line fetches, not fewer).
#include <algorithm>
#include <cstdlib>

#include "sha_core.hpp"

namespace hdrf {


// sha_carry: the 65 dwords (260 B) of four blocks at pos (4-aligned down); the second pair's half
// is carried in registers to the lane's next iteration.  HDRF_SHA_CLAMP (build flag): the 16-B loads
// past the chunk's last byte (end = its END offset) re-read the last one that holds chunk bytes, so a
// chain's final window requests no line beyond the chunk (the padding never reads those bytes:
// pad_block zeroes every word after the message end).
#ifndef HDRF_SHA_CLAMP
#define HDRF_SHA_CLAMP 0
#endif
__device__ __forceinline__ void load_win65(const uint8_t *base, uint64_t readable, uint32_t pos, uint32_t end,
                                           uint32_t d[65])
{
    const uint32_t apos = pos & ~3u;
    if ((uint64_t)apos + 260u <= readable) {
        const HDRF_GLOBAL uint32_t *p = gptr<uint32_t>(base + apos);
        // the last 16-B load with a chunk byte in it (end > pos: the window starts inside the chunk)
        const uint32_t qmax = HDRF_SHA_CLAMP ? (end - 1u - apos) >> 4 : 16u;
#pragma unroll
        for (int q = 0; q < 16; q++) {
            u32x4a v = *(const HDRF_GLOBAL u32x4a *)(p + 4 * min((uint32_t)q, qmax));
            d[4 * q] = v.x; d[4 * q + 1] = v.y; d[4 * q + 2] = v.z; d[4 * q + 3] = v.w;
        }
        d[64] = p[HDRF_SHA_CLAMP ? min(64u, (end - 1u - apos) >> 2) : 64u];
    } else {
#pragma unroll
        for (int q = 0; q < 65; q++) d[q] = load4_guard(base, (int64_t)apos + 4 * q, (int64_t)readable);
    }
}

__device__ __forceinline__ bool pair_at(uint32_t bi, uint32_t T) { return bi < T && ((T - bi) & 1u); }

// The compressions of one iteration from a loaded window (see sha_iter).
template <int HW>
__device__ __forceinline__ void sha_compute(const uint32_t d[33], uint32_t pos, uint32_t len, uint32_t T, uint32_t nb,
                                            uint32_t bi, bool two, uint32_t st[8])
{
    const uint32_t sel = 0x00010203u + (pos & 3u) * 0x01010101u;
    uint32_t m[16];
#pragma unroll
    for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_perm(d[i + 1], d[i], sel);
    if (ballot64(bi >= T)) pad_block(m, len, bi, nb);
    if (HW == 5) sha1_compress(st, m);
    else sha256_compress(st, m);
    if (two) {
#pragma unroll
        for (int i = 0; i < 16; i++) m[i] = __builtin_amdgcn_perm(d[i + 17], d[i + 16], sel);
        if (ballot64(bi + 1 == T)) pad_block(m, len, bi + 1, nb);
        if (HW == 5) sha1_compress(st, m);
        else sha256_compress(st, m);
    }
}

template <int HW>
__device__ __forceinline__ void sha_iter(const uint8_t *base, uint64_t readable, uint32_t s0, uint32_t len, uint32_t T,
                                         uint32_t nb, uint32_t &bi, uint32_t st[8])
{
    const bool two = pair_at(bi, T);
    const uint32_t pos = s0 + 64u * bi;
    uint32_t d[33];
    load_win(base, readable, pos, two, d);
    sha_compute<HW>(d, pos, len, T, nb, bi, two, st);
    bi += two ? 2u : 1u;
}

template <int HW>
__device__ __forceinline__ void store_digest(uint32_t *dst, const uint32_t st[8])
{
#pragma unroll
    for (int i = 0; i < HW; i++) dst[i] = __builtin_bswap32(st[i]);
}

// Long chunks (>= kShaLong bytes: forced cuts of low-entropy runs, up to max_chunk) are hashed by
// dedicated lanes, packed densely.  A chunk's chain is sequential (Merkle-Damgard), so a 1 MB chunk
// keeps its lane busy for 15,625 compressions; left in the per-block queue it sits in a wave whose
// other lanes ran out of chunks, spending a whole SIMD's VALU issue on one lane for tens of
// milliseconds beside the co-running stages (config 4's mixed-entropy blocks hold ~15 % of their
// bytes in such chunks: SHA alone 61 -> 26 ms per batch, config 4 33.5 -> 35.8 GB/s).  The scan
// for them costs config 2 (no long chunks) ~3 %, so the lanes run only while the caller's recent
// batches held long chunks (queue[64], set by the queue consumers whichever mode ran).  The
// workgroups at y = 0 of sha_chunk (dispatched first) scan the offsets of every block (workgroup x
// takes 1024-chunk tiles x, x + gridDim.x, ...), compact the long chunks into LDS and hash them one
// lane each; the queue consumers skip them.  A separate list kernel ahead of sha_chunk cost config 2
// 4 % (one more dependent launch on the SHA stream).
constexpr uint32_t kShaLong = 65536;
constexpr int kShaTile = 1024;                 // chunks per scan tile (4 per thread)

// The long-chunk lanes: workgroups at y = 0 of the SHA grid (see above).
template <int HW>
__device__ __forceinline__ void sha_long_lanes(const BlockDesc *__restrict__ blocks, const uint32_t *__restrict__ offsets,
                                               const BlockState *__restrict__ bst, int cap_blk,
                                               uint32_t *__restrict__ digests, uint32_t thr, int setprio_long)
{
    if (thr == 0xffffffffu) return;
    if (setprio_long) __builtin_amdgcn_s_setprio(3);   // one lane's 15,625-compression chain per 1 MB chunk
    __shared__ uint32_t s_long[kShaTile + 256];
    __shared__ uint32_t s_nl;
    const int t = threadIdx.x;
    if (t == 0) s_nl = 0;
    __syncthreads();
    auto drain = [&]() {                       // every listed chunk: one lane's chain
        const uint32_t nl = s_nl;
        for (uint32_t i = t; i < nl; i += 256) {
            const uint32_t e = s_long[i];
            const int lb = (int)(e >> 26), lk = (int)(e & 0x3ffffffu);   // block < 64, chunk < cap_blk < 2^26
            const uint32_t *lo = offsets + (size_t)lb * cap_blk;
            const uint32_t s0 = lk ? lo[lk - 1] : 0u;
            const uint32_t len = lo[lk] - s0, T = len >> 6, nb = (len + 8) / 64 + 1;
            uint32_t st[8], bi = 0;
            set_iv<HW>(st);
            const BlockDesc &lbd = blocks[lb];
            while (bi < nb) sha_iter<HW>(lbd.data, lbd.readable, s0, len, T, nb, bi, st);
            store_digest<HW>(digests + ((size_t)lb * cap_blk + lk) * HW, st);
        }
        __syncthreads();
        if (t == 0) s_nl = 0;
        __syncthreads();
    };
    const int nblk = (int)gridDim.y - 1;
    for (int lb = 0; lb < nblk; lb++) {
        const int n = bst[lb].n_chunks;
        const uint32_t *lo = offsets + (size_t)lb * cap_blk;
        for (int tb = blockIdx.x * kShaTile; tb < n; tb += gridDim.x * kShaTile) {
            const int k0 = tb + 4 * t;
            uint32_t o[5];
#pragma unroll
            for (int j = 0; j < 5; j++) {
                const int k = k0 - 1 + j;
                o[j] = (k >= 0 && k < n) ? lo[k] : 0u;
            }
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (k0 + j < n && o[j + 1] - o[j] >= thr) s_long[atomicAdd(&s_nl, 1u)] = ((uint32_t)lb << 26) | (uint32_t)(k0 + j);
            __syncthreads();
            const uint32_t cnt = s_nl;
            __syncthreads();
            if (cnt >= 256) drain();          // <= 255 + kShaTile entries at any time
        }
    }
    __syncthreads();
    const uint32_t cnt = s_nl;
    __syncthreads();
    if (cnt) drain();
}

// grid (waves_per_block/4, nblocks + 1): every wave of y = b + 1 serves chunks of block b.  A lane
// owns one chunk's whole compression chain, padding and digest included (the separate tail kernel
// and its mid-state round trip are gone: 1.2 GB of 128-B line fetches per 4 GiB batch, PMC r03).
// Chunk offsets come from coalesced per-wave reservations of 64 chunks kept in registers (pool P,
// with the next reservation Q fetched while P is consumed), so a lane that finishes its chain takes
// the next chunk with two ds_bpermutes and no memory round trip.
template <int HW, bool CARRY>
__device__ __forceinline__ void sha_chunk_body(const BlockDesc *__restrict__ blocks,
                                               const uint32_t *__restrict__ offsets,
                                               const BlockState *__restrict__ bst, int cap_blk,
                                               uint32_t *__restrict__ digests, uint32_t *__restrict__ queue,
                                               uint32_t thr, int prio)
{
    if (blockIdx.y == 0) {                        // the long-chunk lanes (dispatched first)
        sha_long_lanes<HW>(blocks, offsets, bst, cap_blk, digests, thr, prio & 1);
        return;
    }
    if (prio & 2) __builtin_amdgcn_s_setprio(2);        // HDRF_SETPRIO bit 3: the chunk lanes too
    const int b = blockIdx.y - 1;
    const int n = bst[b].n_chunks;
    const BlockDesc &bd = blocks[b];
    const uint8_t *base = bd.data;
    const uint64_t readable = bd.readable;
    const uint32_t *off = offsets + (size_t)b * cap_blk;
    uint32_t *db = digests + (size_t)b * cap_blk * HW;
    const int l = lane_id();
    int kbP, cntP, kbQ, cntQ;
    uint32_t SP, EP, SQ, EQ;
    auto reserve = [&](int &kb, int &cnt, uint32_t &S, uint32_t &E) {
        uint32_t got = 0;
        if (l == 0) got = atomicAdd(queue + b, 64u);
        kb = (int)rdfirst(got);
        cnt = max(0, min(64, n - kb));
        const int k = kb + l;
        E = l < cnt ? ld4(off + k) : 0u;
        S = (l < cnt && k > 0) ? ld4(off + k - 1) : 0u;
    };
    reserve(kbP, cntP, SP, EP);
    reserve(kbQ, cntQ, SQ, EQ);
    int head = 0;
    bool active = false;
    int k = 0;
    uint32_t s0 = 0, len = 0, T = 0, nb = 0, bi = 0;
    uint32_t st[8];
    set_iv<HW>(st);
    uint32_t dw[CARRY ? 65 : 1];                  // sha_carry: the lane's 4-block window
    bool carry = false;                           // its second pair is the lane's next iteration
    for (;;) {
        if (active && bi == nb) {                 // chain done: the digest
            store_digest<HW>(db + (size_t)k * HW, st);
            active = false;
        }
        for (;;) {                                 // offer chunks to idle lanes
            const unsigned long long idle = ballot64(!active);
            if (!idle) break;
            if (head >= cntP) {                   // pool P exhausted: rotate in Q, fetch the next
                if (cntQ == 0) break;
                kbP = kbQ; cntP = cntQ; SP = SQ; EP = EQ; head = 0;
                reserve(kbQ, cntQ, SQ, EQ);
            }
            const int rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0));
            const int avail = cntP - head;
            const int idx = min(head + rank, 63);
            const uint32_t e = (uint32_t)__shfl((int)EP, idx, 64), c0 = (uint32_t)__shfl((int)SP, idx, 64);
            bool skip = false;
            if (ballot64(!active && rank < avail && e - c0 >= kShaLong) && l == 0) atomicOr(queue + 64, 1u);
            if (!active && rank < avail && e - c0 >= thr) {
                skip = true;                      // a long chunk: hashed by the long lanes, take another
            } else if (!active && rank < avail) {
                k = kbP + head + rank;
                s0 = c0;
                len = e - c0;
                T = len >> 6;
                nb = (len + 8) / 64 + 1;
                bi = 0;
                set_iv<HW>(st);
                active = true;
                carry = false;
            }
            const int nidle = __popcll(idle);
            head += min(nidle, avail);
            if (!ballot64(skip) && nidle <= avail) break;
        }
        if (!ballot64(active)) break;
        if constexpr (CARRY) {
            // Lanes alternate: load four blocks (260 B) and run the first pair, then run the second
            // pair from registers (33 moves per four blocks).  Each 128-B line is then shared by two windows once per 256 B of
            // chunk instead of once per 128 B (the 132-B window re-fetches it: 1.41x the bytes).
            if (active) {
                const bool two = pair_at(bi, T);
                const uint32_t pos = s0 + 64u * bi;
                if (carry) {
#pragma unroll
                    for (int i = 0; i < 33; i++) dw[i] = dw[i + 32];
                } else {
                    // four blocks even when the chain has fewer left: a third branch loading only
                    // 132 B for the last pair made the wave wait twice (SHA 2.55 -> 2.85 ms per
                    // batch, profiles/r03_sha_carry_trim_ab.txt)
                    load_win65(base, readable, pos, s0 + len, dw);
                }
                sha_compute<HW>(dw, pos, len, T, nb, bi, two, st);
                carry = !carry && two && bi + 2u < nb;
                bi += two ? 2u : 1u;
            }
        } else {
            if (active) sha_iter<HW>(base, readable, s0, len, T, nb, bi, st);
        }
    }
}

template <int HW>
__global__ void __launch_bounds__(256) sha_chunk_kernel(const BlockDesc *__restrict__ blocks,
                                                        const uint32_t *__restrict__ offsets,
                                                        const BlockState *__restrict__ bst, int cap_blk,
                                                        uint32_t *__restrict__ digests, uint32_t *__restrict__ queue,
                                                        uint32_t thr, int prio)
{
    sha_chunk_body<HW, false>(blocks, offsets, bst, cap_blk, digests, queue, thr, prio);
}

// sha_carry: 4-block windows with the second pair carried in registers.  Round 3 A/B on two boxes:
// +2.0 % and -0.5 % (profiles/r03_sha_carry_ab.txt, r03_sha_carry_ab2.txt); round 5, with sha.hip built
// with uniform regions unstructurized and primed steps: 1136.1 / 1135.2 / 1137.8 vs 1105.2 / 1102.0 /
// 1101.1 GB/s (profiles/r05_carry_ab.txt) — the default since.  HDRF_SHA_CARRY=0: sha_chunk.
template <int HW>
__global__ void __launch_bounds__(256) sha_carry_kernel(const BlockDesc *__restrict__ blocks,
                                                        const uint32_t *__restrict__ offsets,
                                                        const BlockState *__restrict__ bst, int cap_blk,
                                                        uint32_t *__restrict__ digests, uint32_t *__restrict__ queue,
                                                        uint32_t thr, int prio)
{
    sha_chunk_body<HW, true>(blocks, offsets, bst, cap_blk, digests, queue, thr, prio);
}


// The fused front's fix-up (lanehash.hip): the chunks still marked in need[] — each block's last chunk
// (the drop-last rule), a jump target's first, the repair walk's and the sequential fallback's — are
// compacted into a list (block << 26 | chunk), then hashed one lane each.  Config 2 leaves about one
// per block; iterating the per-block queues over every chunk instead cost 0.53 ms per batch.
__global__ void __launch_bounds__(256) need_list_kernel(const BlockState *__restrict__ bst, int cap_blk,
                                                        const uint8_t *__restrict__ need, uint32_t *__restrict__ list,
                                                        uint32_t *__restrict__ count)
{
    const int b = blockIdx.y;
    const int n = bst[b].n_chunks;
    if ((int)blockIdx.x * 1024 >= n) return;
    const int k0 = blockIdx.x * 1024 + 4 * threadIdx.x;
    const uint8_t *nb = need + (size_t)b * cap_blk;
    uint32_t f = 0;
#pragma unroll
    for (int j = 0; j < 4; j++)
        if (k0 + j < n && nb[k0 + j]) f |= 1u << j;
    const uint32_t c = (uint32_t)__popc(f);
    const uint32_t incl = wave_incl_scan(c);
    uint32_t base = 0;
    if (lane_id() == 63 && incl) base = atomicAdd(count, incl);
    base = (uint32_t)__shfl((int)base, 63, 64) + incl - c;
    for (int j = 0; j < 4; j++)
        if (f & (1u << j)) list[base++] = ((uint32_t)b << 26) | (uint32_t)(k0 + j);
}

template <int HW>
__global__ void __launch_bounds__(256) sha_list_kernel(const BlockDesc *__restrict__ blocks,
                                                       const uint32_t *__restrict__ offsets, int cap_blk,
                                                       uint32_t *__restrict__ digests, const uint32_t *__restrict__ list,
                                                       const uint32_t *__restrict__ count)
{
    const uint32_t nl = *count;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nl; i += gridDim.x * 256) {
        const uint32_t e = list[i];
        const int lb = (int)(e >> 26), lk = (int)(e & 0x3ffffffu);
        const uint32_t *lo = offsets + (size_t)lb * cap_blk;
        const uint32_t s0 = lk ? lo[lk - 1] : 0u;
        const uint32_t len = lo[lk] - s0, T = len >> 6, nb = (len + 8) / 64 + 1;
        uint32_t st[8], bi = 0;
        set_iv<HW>(st);
        const BlockDesc &bd = blocks[lb];
        while (bi < nb) sha_iter<HW>(bd.data, bd.readable, s0, len, T, nb, bi, st);
        store_digest<HW>(digests + ((size_t)lb * cap_blk + lk) * HW, st);
    }
}

hipError_t launch_sha_need(int hasher, const BlockDesc *d_blocks, int nblocks, const uint32_t *offsets,
                           const BlockState *bst, int cap_blk, uint32_t *digests, uint32_t *queue, const uint8_t *need,
                           uint32_t *list, hipStream_t st, Marker *mk)
{
    if (nblocks > 64) return hipErrorInvalidValue;
    if (hipError_t e = hipMemsetAsync(queue, 0, sizeof(uint32_t) * 67, st)) return e;
    mk->mark(st);
    const int tiles = (cap_blk + 1023) / 1024;
    hipLaunchKernelGGL(need_list_kernel, dim3(tiles, nblocks), dim3(256), 0, st, bst, cap_blk, need, list, queue + 66);
    if (hasher == 0)
        hipLaunchKernelGGL(sha_list_kernel<5>, dim3(64), dim3(256), 0, st, d_blocks, offsets, cap_blk, digests, list, queue + 66);
    else
        hipLaunchKernelGGL(sha_list_kernel<7>, dim3(64), dim3(256), 0, st, d_blocks, offsets, cap_blk, digests, list, queue + 66);
    mk->mark(st);
    return hipGetLastError();
}

hipError_t launch_sha(int hasher, const BlockDesc *d_blocks, int nblocks, const uint32_t *offsets,
                      const BlockState *bst, int cap_blk, uint32_t *digests, uint32_t *queue, bool long_lanes,
                      hipStream_t st, Marker *mk)
{
    if (nblocks > 64) return hipErrorInvalidValue;
    if (hipError_t e = hipMemsetAsync(queue, 0, sizeof(uint32_t) * 65, st)) return e;
    mk->mark(st);
    // HDRF_SHA_LONG: long-chunk threshold in bytes (>= kShaLong; 0 = no long lanes, for A/B runs)
    // (the caller turns the lanes on while its batches hold long chunks: queue[64], set by sha_chunk)
    static const uint32_t thr_env = [] {
        const char *e = getenv("HDRF_SHA_LONG");
        const long v = e ? atol(e) : (long)kShaLong;
        return v <= 0 ? 0xffffffffu : (uint32_t)std::max<long>(v, kShaLong);
    }();
    const uint32_t thr = long_lanes ? thr_env : 0xffffffffu;
    // 2 waves per SIMD (r02, pipelined with chunking on its own stream: 992 GB/s vs 940 at 3 and
    // 919 at 4) — fewer concurrent per-lane streams thrash L2 less and leave CUs to the
    // co-running place / granule passes; env knobs for
    // experiments: HDRF_SHA_WAVES (waves per SIMD over 1024 SIMDs), HDRF_SHA_LDS (bytes per WG)
    // HDRF_SHA_WPC: waves per CU over the chip's 256 CUs (overrides HDRF_SHA_WAVES x 4)
    static const int per_cu = [] {
        const char *c = getenv("HDRF_SHA_WPC");
        if (c) return atoi(c);
        const char *e = getenv("HDRF_SHA_WAVES");
        return 4 * (e ? atoi(e) : 2);
    }();
    static const int lds = [] { const char *e = getenv("HDRF_SHA_LDS"); return e ? atoi(e) : 0; }();
    // HDRF_SHA_CARRY: 1 = sha_carry (4-block windows, the second pair carried in registers; default),
    // 0 = sha_chunk
    static const bool carryk = [] { const char *e = getenv("HDRF_SHA_CARRY"); return !e || atoi(e) != 0; }();
    const int wpb = std::max(4, (per_cu * 256 / nblocks) & ~3);
    dim3 g(wpb / 4, nblocks + 1);                  // y = 0: the long-chunk lanes
    if (carryk && hasher == 0)
        hipLaunchKernelGGL(sha_carry_kernel<5>, g, dim3(256), lds, st, d_blocks, offsets, bst, cap_blk, digests, queue, thr, (setprio_mask() >> 2) & 3);
    else if (carryk)
        hipLaunchKernelGGL(sha_carry_kernel<7>, g, dim3(256), lds, st, d_blocks, offsets, bst, cap_blk, digests, queue, thr, (setprio_mask() >> 2) & 3);
    else if (hasher == 0)
        hipLaunchKernelGGL(sha_chunk_kernel<5>, g, dim3(256), lds, st, d_blocks, offsets, bst, cap_blk, digests, queue, thr, (setprio_mask() >> 2) & 3);
    else
        hipLaunchKernelGGL(sha_chunk_kernel<7>, g, dim3(256), lds, st, d_blocks, offsets, bst, cap_blk, digests, queue, thr, (setprio_mask() >> 2) & 3);
    mk->mark(st);                                  // (the stage timer's former tail slot: empty)
    return hipGetLastError();
}

}  // namespace hdrf
