// index.hip — GPU-resident fingerprint index with HDRF's exact dedup semantics.
//
// Reference semantics:
//   * index key = digest bytes, value = 11-byte chunkMeta (DN/chunkMeta.java:62-77);
//   * a block's GETs all happen before its SETs (DN/DataDeduplicator.java:588-613 vs
//     :702-818) and blocks are serialised by the FIFO (:124-158,197-204)
//     => chunk is a duplicate  iff  its digest was stored by an EARLIER block;
//   * duplicates inside one block are both "new" (identity HashMap, :338-367);
//   * nCopy = (#distinct blocks holding the digest) mod 256; the location is the one SET by
//     the first block's last occurrence (later SETs re-write the decoded location).
//
// Batched formulation (blocks b = 0..63 of a batch, in arrival order):
//   claim  — probe open addressing by the 8-byte tag; CAS-claim empty slots
//   apply  — verify the full digest; atomicOr(mask, 1<<b); atomicMax(first, (63-b)<<32|k)
//   slow   — single-thread exact re-probe for the (astronomically rare) 8-byte tag collisions
//   decide — is_new = entry created this batch && b == min block; designated = (min block,
//            last chunk index) is the one chunk that writes the final value (in store.hip)
#include <cstdlib>

#include "launchers.hpp"

namespace hdrf {

// Block b holds the digest: set its batch-mask bit.  Only a REPEAT inside one block (the bit was
// already set) records its key in `first` = max((63-b)<<32 | k+1); decide completes the max over
// the minimum block's occurrences when that block has repeats.  One returning atomic per chunk.
__device__ __forceinline__ void record_occurrence(IndexEntry *e, int b, int k)
{
    const unsigned long long bit = 1ull << b;
    const unsigned long long old = atomicOr(&e->mask, bit);
    if (old & bit) atomicMax(&e->first, ((unsigned long long)(63 - b) << 32) | (unsigned)(k + 1));
}

// ---- claim: grid (ceil(cap_blk/256), nblocks) ---------------------------------------------
// Probe by tag; CAS-claim empty slots (an entry of an older epoch is empty: the CAS replaces the
// tag it read).  The chunk's block bit / last occurrence are applied right here when the digest is
// known to match: the claimer (its digest IS the entry's: it initialises the batch-local fields
// with its own occurrence), or an entry created by an earlier batch of this epoch (batch in
// [bfirst, cur): its digest bytes are immutable).  Tag hits on entries created in this batch by
// another lane are deferred to apply (their digest bytes may not be visible yet) — and so is a
// stale `batch` of the previous epoch read between another lane's CAS and its batch store (such
// ids are < bfirst).  flags bit 3 = applied.
template <int HW>
__global__ void __launch_bounds__(256) idx_claim_kernel(const BlockState *__restrict__ bst, int cap_blk,
                                                        const uint32_t *__restrict__ digests,
                                                        IndexEntry *__restrict__ tab, int log2cap, uint32_t cur,
                                                        uint32_t bfirst, unsigned long long key,
                                                        uint32_t *__restrict__ slot, uint8_t *__restrict__ flags,
                                                        int *__restrict__ err)
{
    const int b = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= bst[b].n_chunks) return;
    const size_t c = (size_t)b * cap_blk + k;
    uint32_t dw[HW];
#pragma unroll
    for (int i = 0; i < HW; i++) dw[i] = digests[c * HW + i];
    const unsigned long long tag = tag_word(dw, key);
    const uint64_t mask = (1ull << log2cap) - 1;
    uint64_t h = tag_home(tag, log2cap);
    bool mine = false;
    for (uint64_t probe = 0;; probe++) {
        if (probe > mask) { atomicOr(err, 2); return; }           // table full
        IndexEntry *e = tab + h;
        unsigned long long t = __hip_atomic_load(&e->tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (!tag_live(t, key)) {                                // empty: claim it
            const unsigned long long old = atomicCAS(&e->tag, t, tag);
            if (old == t) { mine = true; break; }
            t = old;
        }
        if (mine) {
            e->batch = cur;
            e->mask = 1ull << b;                                   // this chunk's occurrence
            e->first = 0;
            store_dig<HW>(e, dw);
            break;
        }
        if (t == tag) break;
        h = (h + 1) & mask;
    }
    slot[c] = (uint32_t)h;
    IndexEntry *e = tab + h;
    bool apply = false;
    if (!mine) {
        const uint32_t bt = e->batch;
        apply = bt >= bfirst && bt != cur && entry_matches<HW>(*e, dw);
        if (apply) record_occurrence(e, b, k);
    }
    flags[c] = (mine || apply) ? 8 : 0;
}

// ---- apply: deferred chunks — verify full digest, record block membership / last occurrence
template <int HW>
__global__ void __launch_bounds__(256) idx_apply_kernel(const BlockState *__restrict__ bst, int cap_blk,
                                                        const uint32_t *__restrict__ digests,
                                                        IndexEntry *__restrict__ tab, const uint32_t *__restrict__ slot,
                                                        const uint8_t *__restrict__ flags,
                                                        uint32_t *__restrict__ coll, uint32_t *__restrict__ ncoll,
                                                        int coll_cap, int *__restrict__ err)
{
    const int b = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= bst[b].n_chunks) return;
    const size_t c = (size_t)b * cap_blk + k;
    if (flags[c] & 8) return;
    uint32_t dw[HW];
#pragma unroll
    for (int i = 0; i < HW; i++) dw[i] = digests[c * HW + i];
    IndexEntry *e = tab + slot[c];
    if (entry_matches<HW>(*e, dw)) {
        record_occurrence(e, b, k);
    } else {
        uint32_t i = atomicAdd(ncoll, 1u);
        if ((int)i < coll_cap) coll[i] = (uint32_t)c;
        else atomicOr(err, 4);
    }
}

// ---- slow path: one thread, exact sequential re-probe of tag-collided chunks --------------
template <int HW>
__global__ void idx_slow_kernel(int cap_blk, const uint32_t *__restrict__ digests, IndexEntry *__restrict__ tab,
                                int log2cap, uint32_t cur, unsigned long long key, uint32_t *__restrict__ slot,
                                const uint32_t *__restrict__ coll, const uint32_t *__restrict__ ncoll, int coll_cap,
                                int *__restrict__ err)
{
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t n = min(*ncoll, (uint32_t)coll_cap);
    const uint64_t mask = (1ull << log2cap) - 1;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t c = coll[i];
        const int b = (int)(c / (uint32_t)cap_blk), k = (int)(c % (uint32_t)cap_blk);
        uint32_t dw[HW];
        for (int q = 0; q < HW; q++) dw[q] = digests[(size_t)c * HW + q];
        const unsigned long long tag = tag_word(dw, key);
        uint64_t h = (slot[c] + 1) & mask;
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
        slot[c] = (uint32_t)h;
        IndexEntry *e = tab + h;
        const unsigned long long bit = 1ull << b;
        if (e->mask & bit) {
            const unsigned long long f = ((unsigned long long)(63 - b) << 32) | (unsigned)(k + 1);
            if (f > e->first) e->first = f;
        }
        e->mask |= bit;
    }
}

// ---- decide: is_new / designated + per-tile new-byte sums ---------------------------------
// flags bit0 = is_new, bit1 = in the entry's min block, bit2 = entry created this batch,
// bit4 = the min block repeats the digest (designated = its last occurrence, see place_kernel).  tilesum[b][tile] = sum of new-chunk lengths of the 256 chunks of this workgroup.
__global__ void __launch_bounds__(256) idx_decide_kernel(const BlockState *__restrict__ bst, int cap_blk,
                                                         const uint32_t *__restrict__ offsets,
                                                         IndexEntry *__restrict__ tab,
                                                         const uint32_t *__restrict__ slot, uint32_t cur,
                                                         uint8_t *__restrict__ flags, uint32_t *__restrict__ tilesum,
                                                         int ntiles, uint8_t *__restrict__ dcnt)
{
    __shared__ uint32_t s_part[4];
    const int b = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int n = bst[b].n_chunks;
    uint32_t newlen = 0;
    if (k < n) {
        const size_t c = (size_t)b * cap_blk + k;
        IndexEntry *e = tab + slot[c];
        const unsigned long long m = e->mask;
        const unsigned long long f = e->first;
        const int minb = __builtin_ctzll(m);            // first block of the batch holding it
        const bool created = e->batch == cur;
        const bool is_new = created && b == minb;
        // the min block repeats the digest: every occurrence there joins the max so the
        // designated writer (last occurrence, chunkMeta SET order) is known after this kernel
        const bool rep = b == minb && f != 0 && (63 - (int)(f >> 32)) == minb;
        if (rep) atomicMax(&e->first, ((unsigned long long)(63 - b) << 32) | (unsigned)(k + 1));
        // bit1: in the min block (designated unless it has repeats: resolved in place_kernel)
        // with dcnt (idx_finalize follows): a min-block chunk without repeats is the designated one
        // already — its block count and flag 32 are written here, from the mask this kernel read,
        // so idx_finalize only clears its entry (stores, no line fetch)
        const bool desig_now = dcnt && b == minb && !rep;
        if (desig_now) dcnt[c] = (uint8_t)__popcll(m);
        flags[c] = (uint8_t)((is_new ? 1 : 0) | (b == minb ? 2 : 0) | (created ? 4 : 0) | (rep ? 16 : 0) |
                             (desig_now ? 32 : 0));
        if (is_new) {
            const uint32_t *off = offsets + (size_t)b * cap_blk;
            newlen = off[k] - (k ? off[k - 1] : 0u);
        }
    }
    // workgroup sum of new bytes
    uint32_t v = newlen;
    for (int d = 32; d >= 1; d >>= 1) v += (uint32_t)__shfl_xor((int)v, d, 64);
    if (lane_id() == 0) s_part[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0)
        tilesum[(size_t)b * ntiles + blockIdx.x] = s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

// ---- finalize: the designated chunk of every touched entry, its block count, and the entry's
// batch-local state cleared, right after decide (single-node contexts).  The store stage then needs
// nothing batch-local from the index, so the next batch's claim / apply / decide (stream B) run while
// this batch is placed (stream B2): place writes only the value fields, which the index kernels never
// read.  flags bit 5 = designated; dcnt = popcount(mask) (blocks of the batch holding the digest).
// The designated chunk (min block, last occurrence) is unique per entry, and the other chunks read
// only `first` (to learn they are not designated: after the clear they read 0, which is no chunk's
// k + 1), so its clear cannot change another chunk's answer.
__global__ void __launch_bounds__(256) idx_finalize_kernel(const BlockState *__restrict__ bst, int cap_blk,
                                                           IndexEntry *__restrict__ tab,
                                                           const uint32_t *__restrict__ slot,
                                                           uint8_t *__restrict__ flags, uint8_t *__restrict__ dcnt)
{
    const int b = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= bst[b].n_chunks) return;
    const size_t c = (size_t)b * cap_blk + k;
    const uint8_t f = flags[c];
    if (!(f & 2)) return;                              // not in the entry's min block
    IndexEntry *e = tab + slot[c];
    if (!(f & 32)) {                                   // not settled by idx_decide:
        if ((f & 16) && (uint32_t)e->first != (uint32_t)(k + 1)) return;   // repeats: the last occurrence
        dcnt[c] = (uint8_t)__popcll(e->mask);
        flags[c] = f | 32;
    }
    e->mask = 0;                                       // (designated without repeats: decided in
    e->first = 0;                                      //  idx_decide, no read of the entry here)
}

hipError_t launch_index_finalize(const BlockState *bst, int nblocks, int cap_blk, int ntiles, IndexEntry *tab,
                                 const uint32_t *slot, uint8_t *flags, uint8_t *dcnt, hipStream_t st)
{
    hipLaunchKernelGGL(idx_finalize_kernel, dim3(ntiles, nblocks), dim3(256), 0, st, bst, cap_blk, tab, slot, flags, dcnt);
    return hipGetLastError();
}

// A fresh DataNode (empty Redis): zero the table with 16-B streaming stores (rocclr's fill
// reached ~1 TB/s on the 8.6 GB table) and seed the allocator, both on the stream that owns
// the index, so the front half of the next batch overlaps the clear.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// ring_per > 0 (a fresh generation of a durable-container context, hdrf_reset_async): the new
// generation's allocator keeps every storer range's slot ring where the old one left it, one slot
// past an open container, so no slot the old generation may still hand out (drain) is reopened
// before the ring comes round to it (the host's ring check counts that slot until the switch).
__global__ void __launch_bounds__(256) idx_clear_kernel(u32x4 *__restrict__ p, uint64_t n16, AllocState *alloc,
                                                        AllocState a, uint32_t ring_per)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (; i + 3 * stride < n16; i += 4 * stride) {
        __builtin_nontemporal_store(z, p + i);
        __builtin_nontemporal_store(z, p + i + stride);
        __builtin_nontemporal_store(z, p + i + 2 * stride);
        __builtin_nontemporal_store(z, p + i + 3 * stride);
    }
    for (; i < n16; i += stride) __builtin_nontemporal_store(z, p + i);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (ring_per)
            for (int t = 0; t < 4; t++) {
                const uint32_t base = (uint32_t)t * ring_per, s = alloc->slot[t];
                a.slot[t] = alloc->exists[t] ? base + (s - base + 1) % ring_per : s;
            }
        *alloc = a;
    }
}

// Restore (a Redis dump of the index: digest -> 11-byte chunkMeta value): one thread per entry,
// claim the first empty slot of the digest's probe sequence, then fill the entry at rest (no
// batch-local state; batch 0 precedes every batch the context will run).  Digests are unique.
template <int HW>
__global__ void __launch_bounds__(256) idx_load_kernel(const uint32_t *__restrict__ dw_all,
                                                       const uint8_t *__restrict__ vals, int n,
                                                       IndexEntry *__restrict__ tab, int log2cap,
                                                       unsigned long long key, uint32_t bload, int *__restrict__ err)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    uint32_t dw[HW];
#pragma unroll
    for (int i = 0; i < HW; i++) dw[i] = dw_all[(size_t)k * HW + i];
    const unsigned long long tag = tag_word(dw, key);
    const uint64_t mask = (1ull << log2cap) - 1;
    uint64_t h = tag_home(tag, log2cap);
    for (uint64_t probe = 0; probe <= mask; probe++, h = (h + 1) & mask) {
        unsigned long long t = tab[h].tag;
        bool mine = false;
        while (!tag_live(t, key)) {
            const unsigned long long old = atomicCAS(&tab[h].tag, t, tag);
            if (old == t) { mine = true; break; }
            t = old;
        }
        if (!mine) continue;
        IndexEntry &e = tab[h];
        const uint8_t *v = vals + (size_t)k * 11;           // chunkMeta.process, DN/chunkMeta.java:35-60
        e.mask = 0;
        e.first = 0;
        e.batch = bload;                                    // a batch before every batch that follows
        e.ncopy = v[0] | (HW == 7 ? (dw[1] >> 24) << 8 : 0u);
        e.cid = ((uint32_t)v[1] << 16) | ((uint32_t)v[2] << 8) | v[3];
        e.start = ((uint32_t)v[4] << 16) | ((uint32_t)v[5] << 8) | v[6] | ((uint32_t)(v[10] & 0xF0) << 20);
        e.stop = ((uint32_t)v[7] << 16) | ((uint32_t)v[8] << 8) | v[9] | ((uint32_t)(v[10] & 0x0F) << 24);
#pragma unroll
        for (int i = 2; i < HW; i++) e.dig[i - 2] = dw[i];
        if (HW == 5) { e.dig[3] = dw[0]; e.dig[4] = dw[1]; }
        return;
    }
    atomicOr(err, 2);                                       // table full
}

hipError_t launch_index_load(int hasher, const uint32_t *dw, const uint8_t *vals, int n, IndexEntry *tab, int log2cap,
                             unsigned long long key, uint32_t bload, int *err, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    const dim3 g((n + 255) / 256);
    if (hasher == 0)
        hipLaunchKernelGGL(idx_load_kernel<5>, g, dim3(256), 0, st, dw, vals, n, tab, log2cap, key, bload, err);
    else
        hipLaunchKernelGGL(idx_load_kernel<7>, g, dim3(256), 0, st, dw, vals, n, tab, log2cap, key, bload, err);
    return hipGetLastError();
}

// Probe lengths of a completed batch (steady-state measurement): each chunk's final slot minus its
// home slot, summed / maxed into stats[0] (sum), stats[1] (max), stats[2] (chunks)
template <int HW>
__global__ void __launch_bounds__(256) idx_probe_kernel(const BlockState *__restrict__ bst, int cap_blk,
                                                        const uint32_t *__restrict__ digests, const uint32_t *__restrict__ slot,
                                                        int log2cap, unsigned long long key,
                                                        unsigned long long *__restrict__ stats)
{
    const int b = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    const bool on = k < bst[b].n_chunks;
    unsigned long long d = 0;
    if (on) {
        const size_t c = (size_t)b * cap_blk + k;
        uint32_t dw[HW];
#pragma unroll
        for (int i = 0; i < HW; i++) dw[i] = digests[c * HW + i];
        const uint64_t mask = (1ull << log2cap) - 1;
        d = ((uint64_t)slot[c] - tag_home(tag_word(dw, key), log2cap)) & mask;
    }
    // wave reductions, one atomic per wave
    unsigned long long s = d, m = d, n = on ? 1ull : 0ull;
    for (int o = 32; o > 0; o >>= 1) {
        s += __shfl_xor(s, o, 64);
        m = max(m, (unsigned long long)__shfl_xor(m, o, 64));
        n += __shfl_xor(n, o, 64);
    }
    if (lane_id() == 0 && n) {
        atomicAdd(&stats[0], s);
        atomicMax(&stats[1], m);
        atomicAdd(&stats[2], n);
    }
}

hipError_t launch_index_probe(int hasher, const BlockState *bst, int nblocks, int cap_blk, const uint32_t *digests,
                              const uint32_t *slot, int log2cap, unsigned long long tag_mask,
                              unsigned long long *stats, hipStream_t st)
{
    dim3 g((cap_blk + 255) / 256, nblocks);
    if (hasher == 0) hipLaunchKernelGGL(idx_probe_kernel<5>, g, dim3(256), 0, st, bst, cap_blk, digests, slot, log2cap, tag_mask, stats);
    else hipLaunchKernelGGL(idx_probe_kernel<7>, g, dim3(256), 0, st, bst, cap_blk, digests, slot, log2cap, tag_mask, stats);
    return hipGetLastError();
}

hipError_t launch_index_clear(IndexEntry *tab, int log2cap, AllocState *d_alloc, const AllocState &a, hipStream_t st,
                              uint32_t ring_per)
{
    // log2cap < 0: seed the allocator only (a reset that bumps the index epoch)
    const uint64_t n16 = log2cap < 0 ? 0 : (sizeof(IndexEntry) << log2cap) / 16;
    uint64_t g = (n16 + 255) / 256;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    hipLaunchKernelGGL(idx_clear_kernel, dim3((unsigned)g), dim3(256), 0, st, (u32x4 *)tab, n16, d_alloc, a, ring_per);
    return hipGetLastError();
}

hipError_t launch_index(int hasher, const BlockState *bst, int nblocks, int cap_blk, const uint32_t *offsets,
                        const uint32_t *digests, IndexEntry *tab, int log2cap, uint32_t cur, uint32_t bfirst,
                        unsigned long long tag_mask, uint32_t *slot,
                        uint32_t *coll, uint32_t *ncoll, int coll_cap, uint8_t *flags, uint32_t *tilesum,
                        int ntiles, int *err, hipStream_t st, Marker *mk, uint8_t *dcnt)
{
    mk->mark(st);
    dim3 g(ntiles, nblocks);
    static const int lds = [] { const char *e = getenv("HDRF_CLAIM_LDS"); return e ? atoi(e) : 0; }();
    if (hipError_t e = hipMemsetAsync(ncoll, 0, sizeof(uint32_t), st)) return e;
    if (hasher == 0) {
        hipLaunchKernelGGL(idx_claim_kernel<5>, g, dim3(256), lds, st, bst, cap_blk, digests, tab, log2cap, cur, bfirst,
                           tag_mask, slot, flags, err);
        mk->mark(st);
        hipLaunchKernelGGL(idx_apply_kernel<5>, g, dim3(256), 0, st, bst, cap_blk, digests, tab, slot, flags, coll,
                           ncoll,
                           coll_cap, err);
        mk->mark(st);
        hipLaunchKernelGGL(idx_slow_kernel<5>, dim3(1), dim3(64), 0, st, cap_blk, digests, tab, log2cap, cur, tag_mask, slot,
                           coll, ncoll, coll_cap, err);
    } else {
        hipLaunchKernelGGL(idx_claim_kernel<7>, g, dim3(256), lds, st, bst, cap_blk, digests, tab, log2cap, cur, bfirst,
                           tag_mask, slot, flags, err);
        mk->mark(st);
        hipLaunchKernelGGL(idx_apply_kernel<7>, g, dim3(256), 0, st, bst, cap_blk, digests, tab, slot, flags, coll,
                           ncoll,
                           coll_cap, err);
        mk->mark(st);
        hipLaunchKernelGGL(idx_slow_kernel<7>, dim3(1), dim3(64), 0, st, cap_blk, digests, tab, log2cap, cur, tag_mask, slot,
                           coll, ncoll, coll_cap, err);
    }
    hipLaunchKernelGGL(idx_decide_kernel, g, dim3(256), 0, st, bst, cap_blk, offsets, tab, slot, cur, flags, tilesum,
                       ntiles, dcnt);
    return hipGetLastError();
}

}  // namespace hdrf
