// gx.hip — node-global fingerprint index across G GPUs (BASELINE config 3).
//
// Reference deployment this reproduces: every DataNode of one host talks to the SAME Redis on
// localhost (DN/DataDeduplicator.java:119), the same "blockID" allocator key (:165-172, :389),
// the same chunkDir and the same static FIFO (:124-158, :197-204).  The node therefore behaves
// as ONE reduction over the global block sequence; G GPUs must give byte-identical decisions,
// index values and container placement to a single sequential run (the oracle).
//
// Per global batch (G ranks x B local blocks, rank r holding batch positions [gbase, gbase+B)):
//   front   (source)  chunk + SHA (chunk.hip, sha.hip), then a LOCAL aggregation of the batch's
//                     digests in a scratch table (index.hip kernels): one record per distinct
//                     digest = (digest, first local batch position holding it, #local blocks
//                     holding it), bucketed by owner rank = first digest word mod G   [gx_emit]
//   X1      all-to-all of records to their owners (RCCL over xGMI, host side)
//   owner   claim/apply/slow the records into the owner's partition of the global index;
//           per entry max(~gpos) = minimum block holding it, sum of counts = new nCopy  [own_*]
//   X2      all-to-all of (owner slot, created, holds-minimum) back to the sources
//   decide  (source) per-chunk is_new / designated flags + new-byte tile sums        [gx_decide]
//   flush   container flush walk, chained rank 0 -> G-1 over the allocator state (store.hip)
//   place   (source) container placement + gather; the designated chunk of each NEW entry
//           emits (owner slot, container id, start, stop)                          [store.hip]
//   X3      all-to-all of those locations; owners commit them                        [own_commit]
#include <algorithm>

#include "launchers.hpp"

namespace hdrf {

__device__ __forceinline__ int owner_of(uint32_t dw0, int G) { return (int)(dw0 % (uint32_t)G); }

// ---- gx_emit: grid (ceil(ntiles / kEmitTiles), nblocks) over the local batch -----------------
// The chunk designated in the scratch table (min local block, its last occurrence) emits the
// digest's record.  scratch.cid <- response index (owner * cap + i).  A workgroup takes kEmitTiles
// tiles of 256 chunks and reserves its records with one atomic per owner (wg_reserve): one atomic
// per record on the G counters serialised at the memory side (30.8 ms per 4 GiB batch, one per
// wave still 1.5 ms; profiles/r06_lb2_kernel_stats.csv, r06_lb2b_kernel_stats.csv).
constexpr int kEmitTiles = 4;
template <int HW>
__global__ void __launch_bounds__(256) gx_emit_kernel(const BlockState *__restrict__ bst, int cap_blk,
                                                      const uint32_t *__restrict__ digests,
                                                      IndexEntry *__restrict__ scratch, const uint32_t *__restrict__ slot,
                                                      const uint8_t *__restrict__ flags, uint32_t gbase, int G,
                                                      uint32_t *__restrict__ x1, int64_t cap,
                                                      unsigned long long *__restrict__ counts, int *__restrict__ err)
{
    __shared__ uint32_t s_cnt[64];
    __shared__ unsigned long long s_base[64];
    const int b = blockIdx.y, t = (int)threadIdx.x;
    const int n = bst[b].n_chunks;
    if ((int)blockIdx.x * kEmitTiles * 256 >= n) return;     // (uniform)
    if (t < G) s_cnt[t] = 0u;
    __syncthreads();
    bool want[kEmitTiles];
    int dd[kEmitTiles];
    uint32_t li[kEmitTiles];
#pragma unroll
    for (int j = 0; j < kEmitTiles; j++) {
        const int k = ((int)blockIdx.x * kEmitTiles + j) * 256 + t;
        want[j] = false;
        dd[j] = 0;
        li[j] = 0;
        if (k < n) {
            const size_t c = (size_t)b * cap_blk + k;
            const uint8_t f = flags[c];
            // in the digest's min local block, and its last occurrence there
            if ((f & 2) && (!(f & 16) || (uint32_t)scratch[slot[c]].first == (uint32_t)(k + 1))) {
                want[j] = true;
                dd[j] = owner_of(digests[c * HW], G);
                li[j] = atomicAdd(&s_cnt[dd[j]], 1u);
            }
        }
    }
    __syncthreads();
    if (t < G && s_cnt[t]) s_base[t] = atomicAdd(counts + t, (unsigned long long)s_cnt[t]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kEmitTiles; j++) {
        if (!want[j]) continue;
        const int k = ((int)blockIdx.x * kEmitTiles + j) * 256 + t;
        const size_t c = (size_t)b * cap_blk + k;
        const int d = dd[j];
        const unsigned long long i = s_base[d] + li[j];
        if ((int64_t)i >= cap) { atomicOr(err, 16); continue; }
        IndexEntry *e = scratch + slot[c];
        uint32_t *rec = x1 + ((size_t)d * cap + i) * (HW + 2);
#pragma unroll
        for (int q = 0; q < HW; q++) rec[q] = digests[c * HW + q];
        rec[HW] = gbase + (uint32_t)b;                          // batch position of the min block
        rec[HW + 1] = (uint32_t)__popcll(e->mask);              // local blocks holding the digest
        e->cid = (uint32_t)((size_t)d * cap + i);
    }
}

// ---- owner side: grid (ceil(cap/256), G) over the records received from each source ------
// IndexEntry fields during a batch: first = max over records of ~gpos (-> min block), mask =
// sum of counts (-> blocks holding the digest this batch); both reset by own_finish.
__device__ __forceinline__ void own_record(IndexEntry *e, uint32_t gpos, uint32_t cnt)
{
    atomicMax(&e->first, (unsigned long long)(0xffffffffu - gpos));
    atomicAdd(&e->mask, (unsigned long long)cnt);
}

// oflags bit 3 = applied in claim
// (claim rules as index.hip idx_claim_kernel: epoch-empty entries are claimed by CAS on the tag read,
// the claimer initialises the batch-local fields with its own record, entries of earlier batches of
// this epoch are applied at once, the rest deferred)
template <int HW>
__global__ void __launch_bounds__(256) own_claim_kernel(const uint32_t *__restrict__ x1, const int64_t *__restrict__ counts,
                                                        int64_t cap, IndexEntry *__restrict__ tab, int log2cap,
                                                        uint32_t cur, uint32_t bfirst, unsigned long long key,
                                                        uint32_t *__restrict__ oslot, uint8_t *__restrict__ oflags,
                                                        int *__restrict__ err)
{
    const int s = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= counts[s]) return;
    const size_t r = (size_t)s * cap + i;
    const uint32_t *rec = x1 + r * (HW + 2);
    uint32_t dw[HW];
#pragma unroll
    for (int q = 0; q < HW; q++) dw[q] = rec[q];
    const unsigned long long tag = tag_word(dw, key);
    const uint64_t mask = (1ull << log2cap) - 1;
    uint64_t h = tag_home(tag, log2cap);
    bool mine = false;
    for (uint64_t probe = 0;; probe++) {
        if (probe > mask) { atomicOr(err, 2); return; }
        IndexEntry *e = tab + h;
        unsigned long long t = __hip_atomic_load(&e->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (!tag_live(t, key)) {
            const unsigned long long old = atomicCAS(&e->tag, t, tag);
            if (old == t) { mine = true; break; }
            t = old;
        }
        if (mine) {
            e->batch = cur;
            e->first = (unsigned long long)(0xffffffffu - rec[HW]);    // this record (own_record)
            e->mask = (unsigned long long)rec[HW + 1];
            store_dig<HW>(e, dw);
            break;
        }
        if (t == tag) break;
        h = (h + 1) & mask;
    }
    oslot[r] = (uint32_t)h;
    IndexEntry *e = tab + h;
    bool apply = false;
    if (!mine) {
        const uint32_t bt = e->batch;
        apply = bt >= bfirst && bt != cur && entry_matches<HW>(*e, dw);
        if (apply) own_record(e, rec[HW], rec[HW + 1]);
    }
    oflags[r] = (mine || apply) ? 8 : 0;
}

template <int HW>
__global__ void __launch_bounds__(256) own_apply_kernel(const uint32_t *__restrict__ x1, const int64_t *__restrict__ counts,
                                                        int64_t cap, IndexEntry *__restrict__ tab,
                                                        const uint32_t *__restrict__ oslot, const uint8_t *__restrict__ oflags,
                                                        uint32_t *__restrict__ coll,
                                                        uint32_t *__restrict__ ncoll, int coll_cap, int *__restrict__ err)
{
    const int s = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= counts[s]) return;
    const size_t r = (size_t)s * cap + i;
    if (oflags[r] & 8) return;
    const uint32_t *rec = x1 + r * (HW + 2);
    uint32_t dw[HW];
#pragma unroll
    for (int q = 0; q < HW; q++) dw[q] = rec[q];
    IndexEntry *e = tab + oslot[r];
    if (entry_matches<HW>(*e, dw)) {
        own_record(e, rec[HW], rec[HW + 1]);
    } else {
        const uint32_t j = atomicAdd(ncoll, 1u);
        if ((int)j < coll_cap) coll[j] = (uint32_t)r;
        else atomicOr(err, 4);
    }
}

// exact sequential re-probe of 8-byte tag collisions (one thread)
template <int HW>
__global__ void own_slow_kernel(const uint32_t *__restrict__ x1, IndexEntry *__restrict__ tab, int log2cap, uint32_t cur,
                                unsigned long long key, uint32_t *__restrict__ oslot,
                                const uint32_t *__restrict__ coll, const uint32_t *__restrict__ ncoll, int coll_cap,
                                int *__restrict__ err)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t n = min(*ncoll, (uint32_t)coll_cap);
    const uint64_t mask = (1ull << log2cap) - 1;
    for (uint32_t j = 0; j < n; j++) {
        const size_t r = coll[j];
        const uint32_t *rec = x1 + r * (HW + 2);
        uint32_t dw[HW];
        for (int q = 0; q < HW; q++) dw[q] = rec[q];
        const unsigned long long tag = tag_word(dw, key);
        uint64_t h = (oslot[r] + 1) & mask;
        for (uint64_t probe = 0;; probe++) {
            if (probe > mask) { *err |= 2; return; }
            IndexEntry *e = tab + h;
            if (!tag_live(e->tag, key)) {
                e->tag = tag; e->batch = cur; e->mask = 0; e->first = 0;
                store_dig<HW>(e, dw);
                break;
            }
            if (e->tag == tag && entry_matches<HW>(*e, dw)) break;
            h = (h + 1) & mask;
        }
        oslot[r] = (uint32_t)h;
        IndexEntry *e = tab + h;
        const unsigned long long key = 0xffffffffu - rec[HW];
        if (key > e->first) e->first = key;
        e->mask += rec[HW + 1];
    }
}

// response per record: {owner slot, bit0 created this batch, bit1 record holds the minimum block}.
// The record holding the minimum block (exactly one per entry) finalises nCopy; when the entry was
// created this batch its source will send one X3 location (its designated chunk), counted per source
// in x3exp (the X3 receive counts, no exchange needed).
// After a claim error (table full: a record's oslot was never written; collision list overflow:
// its oslot names an entry holding another digest) no record touches the table again: every
// response is "not created, not the minimum" so the sources designate nothing and send no X3
// location, and the error is reported by hdrf_gx_place.
__global__ void __launch_bounds__(256) own_decide_kernel(const uint32_t *__restrict__ x1, int rw,
                                                         const int64_t *__restrict__ counts, int64_t cap,
                                                         IndexEntry *__restrict__ tab, const uint32_t *__restrict__ oslot,
                                                         uint32_t cur, uint32_t *__restrict__ x2,
                                                         unsigned long long *__restrict__ x3exp, const int *__restrict__ err)
{
    __shared__ uint32_t s_n;
    const int s = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t cnt_s = counts[s];
    if ((int64_t)blockIdx.x * 256 >= cnt_s) return;          // (uniform)
    if (threadIdx.x == 0) s_n = 0u;
    __syncthreads();
    bool want3 = false;
    if (i < cnt_s) {
        const size_t r = (size_t)s * cap + i;
        if (*err & 6) {
            x2[2 * r] = 0;
            x2[2 * r + 1] = 0;
        } else {
            const uint32_t gpos = x1[r * rw + rw - 2];
            const uint32_t h = oslot[r];
            IndexEntry *e = tab + h;
            const bool created = e->batch == cur;
            const bool holds = (uint32_t)e->first == 0xffffffffu - gpos;
            if (holds) {
                const uint32_t cnt = (uint32_t)e->mask;
                // chunkMeta.process: nCopy = old + 1 per later block (DN/chunkMeta.java:35-60), 1 when new
                set_ncopy(e, created ? cnt : e->ncopy + cnt);
            }
            x2[2 * r] = h;
            x2[2 * r + 1] = (created ? 1u : 0u) | (holds ? 2u : 0u);
            want3 = created && holds;
        }
    }
    // the X3 records this owner will receive from source s: one atomic per workgroup
    const unsigned long long m3 = ballot64(want3);
    if (lane_id() == 0 && m3) atomicAdd(&s_n, (uint32_t)__popcll(m3));
    __syncthreads();
    if (threadIdx.x == 0 && s_n) atomicAdd(x3exp + s, (unsigned long long)s_n);
}

__global__ void __launch_bounds__(256) own_finish_kernel(const uint32_t *__restrict__ x2, const int64_t *__restrict__ counts,
                                                         int64_t cap, IndexEntry *__restrict__ tab, const int *__restrict__ err)
{
    const int s = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= counts[s] || (*err & 6)) return;
    const size_t r = (size_t)s * cap + i;
    if (x2[2 * r + 1] & 2) {
        IndexEntry *e = tab + x2[2 * r];
        e->first = 0;
        e->mask = 0;
    }
}

// ---- source: per-chunk decisions from the owners' responses -------------------------------
// flags: bit0 is_new, bit1 in the digest's GLOBAL min block, bit2 created this batch, bit4 that
// block repeats the digest (designated = last occurrence, scratch.first); tilesum as decide.
__global__ void __launch_bounds__(256) gx_decide_kernel(const BlockState *__restrict__ bst, int cap_blk,
                                                        const uint32_t *__restrict__ offsets,
                                                        const IndexEntry *__restrict__ scratch,
                                                        const uint32_t *__restrict__ slot, const uint32_t *__restrict__ x2,
                                                        uint8_t *__restrict__ flags, uint32_t *__restrict__ tilesum,
                                                        int ntiles)
{
    __shared__ uint32_t s_part[4];
    const int b = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int n = bst[b].n_chunks;
    uint32_t newlen = 0;
    if (k < n) {
        const size_t c = (size_t)b * cap_blk + k;
        const uint8_t f = flags[c];
        const uint32_t ri = scratch[slot[c]].cid;
        const uint32_t rf = x2[2 * (size_t)ri + 1];
        const bool created = rf & 1, holds = (rf & 2) && (f & 2);
        const bool is_new = created && holds;
        flags[c] = (uint8_t)((is_new ? 1 : 0) | (holds ? 2 : 0) | (created ? 4 : 0) | (f & 16));
        if (is_new) {
            const uint32_t *off = offsets + (size_t)b * cap_blk;
            newlen = off[k] - (k ? off[k - 1] : 0u);
        }
    }
    uint32_t v = newlen;
    for (int d = 32; d >= 1; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d, 64);
    if (lane_id() == 0) s_part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0)
        tilesum[(size_t)b * ntiles + blockIdx.x] = s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

// ---- source: X3 records this rank must send each owner = the responses "created, holds the
// minimum" it received (one designated chunk per such record emits one location).  place_kernel's
// own counts are checked against these, so a sender whose X3 counts disagree with the owners' X2
// answers (which the owners count for their receive side, own_decide) fails at hdrf_gx_place.
// grid (ceil(max sent / 256), G)
__global__ void __launch_bounds__(256) gx_x3want_kernel(const uint32_t *__restrict__ x2,
                                                        const unsigned long long *__restrict__ sent, int64_t cap,
                                                        unsigned long long *__restrict__ want)
{
    __shared__ uint32_t s_n;
    const int d = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if ((int64_t)blockIdx.x * 256 >= (int64_t)sent[d]) return;   // (uniform)
    if (threadIdx.x == 0) s_n = 0u;
    __syncthreads();
    const bool ok = i < (int64_t)sent[d] && (x2[2 * ((size_t)d * cap + i) + 1] & 3u) == 3u;
    const unsigned long long m = ballot64(ok);
    if (lane_id() == 0 && m) atomicAdd(&s_n, (uint32_t)__popcll(m));   // one global atomic per workgroup
    __syncthreads();
    if (threadIdx.x == 0 && s_n) atomicAdd(want + d, (unsigned long long)s_n);
}

hipError_t launch_gx_x3want(const uint32_t *x2, const unsigned long long *sent, int64_t max_sent, int64_t cap, int G,
                            unsigned long long *want, hipStream_t st)
{
    if (hipError_t e = hipMemsetAsync(want, 0, sizeof(unsigned long long) * G, st)) return e;
    hipLaunchKernelGGL(gx_x3want_kernel, dim3(std::max<int64_t>(1, (max_sent + 255) / 256), G), dim3(256), 0, st, x2,
                       sent, cap, want);
    return hipGetLastError();
}

// ---- owner: commit locations of entries created this batch (X3) ---------------------------
__global__ void __launch_bounds__(256) own_commit_kernel(const uint32_t *__restrict__ x3, const int64_t *__restrict__ counts,
                                                         int64_t cap, IndexEntry *__restrict__ tab, uint64_t tab_n,
                                                         int *__restrict__ err)
{
    const int s = blockIdx.y;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= counts[s]) return;
    const uint32_t *rec = x3 + ((size_t)s * cap + i) * 4;
    if (rec[0] >= tab_n) { atomicOr(err, 256); return; }    // a peer's malformed location: never write outside
    IndexEntry *e = tab + rec[0];
    e->cid = rec[1] | ((uint32_t)(s + 1) << 24);          // ids are < 2^24: bits 24-31 = placing rank + 1
    e->start = rec[2];
    e->stop = rec[3];
}

// ---- host launchers ------------------------------------------------------------------------
static inline unsigned gx_tiles(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + 255) / 256); }

hipError_t launch_gx_emit(int hasher, const BlockState *bst, int nblocks, int cap_blk, int ntiles,
                          const uint32_t *digests, IndexEntry *scratch, const uint32_t *slot, const uint8_t *flags,
                          uint32_t gbase, int G, uint32_t *x1, int64_t cap, unsigned long long *counts, int *err,
                          hipStream_t st)
{
    if (hipError_t e = hipMemsetAsync(counts, 0, sizeof(unsigned long long) * G, st)) return e;
    dim3 g((ntiles + kEmitTiles - 1) / kEmitTiles, nblocks);
    if (hasher == 0)
        hipLaunchKernelGGL(gx_emit_kernel<5>, g, dim3(256), 0, st, bst, cap_blk, digests, scratch, slot, flags, gbase, G,
                           x1, cap, counts, err);
    else
        hipLaunchKernelGGL(gx_emit_kernel<7>, g, dim3(256), 0, st, bst, cap_blk, digests, scratch, slot, flags, gbase, G,
                           x1, cap, counts, err);
    return hipGetLastError();
}

hipError_t launch_gx_owner(int hasher, const uint32_t *x1, const int64_t *counts, int64_t max_count, int64_t cap, int G,
                           IndexEntry *tab, int log2cap, uint32_t cur, uint32_t bfirst, unsigned long long tag_mask, uint32_t *oslot,
                           uint8_t *oflags, uint32_t *coll, uint32_t *ncoll, int coll_cap, uint32_t *x2,
                           unsigned long long *x3exp, int *err, hipStream_t st)
{
    const int HW = hasher == 0 ? 5 : 7;
    dim3 g(gx_tiles(max_count), G);
    if (hipError_t e = hipMemsetAsync(ncoll, 0, sizeof(uint32_t), st)) return e;
    if (hasher == 0) {
        hipLaunchKernelGGL(own_claim_kernel<5>, g, dim3(256), 0, st, x1, counts, cap, tab, log2cap, cur, bfirst, tag_mask,
                           oslot, oflags, err);
        hipLaunchKernelGGL(own_apply_kernel<5>, g, dim3(256), 0, st, x1, counts, cap, tab, oslot, oflags, coll,
                           ncoll, coll_cap, err);
        hipLaunchKernelGGL(own_slow_kernel<5>, dim3(1), dim3(64), 0, st, x1, tab, log2cap, cur, tag_mask, oslot, coll,
                           ncoll, coll_cap, err);
    } else {
        hipLaunchKernelGGL(own_claim_kernel<7>, g, dim3(256), 0, st, x1, counts, cap, tab, log2cap, cur, bfirst, tag_mask,
                           oslot, oflags, err);
        hipLaunchKernelGGL(own_apply_kernel<7>, g, dim3(256), 0, st, x1, counts, cap, tab, oslot, oflags, coll,
                           ncoll, coll_cap, err);
        hipLaunchKernelGGL(own_slow_kernel<7>, dim3(1), dim3(64), 0, st, x1, tab, log2cap, cur, tag_mask, oslot, coll,
                           ncoll, coll_cap, err);
    }
    hipLaunchKernelGGL(own_decide_kernel, g, dim3(256), 0, st, x1, HW + 2, counts, cap, tab, oslot, cur, x2, x3exp, err);
    hipLaunchKernelGGL(own_finish_kernel, g, dim3(256), 0, st, x2, counts, cap, tab, err);
    return hipGetLastError();
}

hipError_t launch_gx_decide(const BlockState *bst, int nblocks, int cap_blk, int ntiles, const uint32_t *offsets,
                            const IndexEntry *scratch, const uint32_t *slot, const uint32_t *x2, uint8_t *flags,
                            uint32_t *tilesum, hipStream_t st)
{
    hipLaunchKernelGGL(gx_decide_kernel, dim3(ntiles, nblocks), dim3(256), 0, st, bst, cap_blk, offsets, scratch, slot, x2,
                       flags, tilesum, ntiles);
    return hipGetLastError();
}

hipError_t launch_gx_commit(const uint32_t *x3, const int64_t *counts, int64_t max_count, int64_t cap, int G,
                            IndexEntry *tab, int log2cap, int *err, hipStream_t st)
{
    hipLaunchKernelGGL(own_commit_kernel, dim3(gx_tiles(max_count), G), dim3(256), 0, st, x3, counts, cap, tab,
                       (uint64_t)1 << log2cap, err);
    return hipGetLastError();
}

}  // namespace hdrf
