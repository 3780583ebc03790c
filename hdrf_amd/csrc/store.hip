// store.hip — container placement, gather and index finalisation on gfx950.
//
// Reference: threadedStorer.run, DN/DataDeduplicator.java:702-836 (driver storeChunksMT
// :511-532).  Storer t owns chunk range [n*t/3, n*(t+1)/3) (1 range when n < 25) and the
// container lastBlockID[t]; it appends each NEW chunk at curPos, and when
// curPos + len > maxSize it closes the container (rewritten whole, :748-786), bumps the id and
// restarts at 0 (:790-796).  The open container's tail is appended raw (:806-818) and
// lastBlockID[t+4] = bytes appended by this block since its last flush (:808).  A block with
// storeSize == 0 touches no container (:713-719).
//
// Because every storer t only ever appends to its own container chain, the placement of all
// new chunks of a batch is a prefix sum per range plus a short sequential walk over the
// flush points (each found with a 64-ary search over the prefix array):
//   tile_scan   — per block: exclusive scan of the per-tile new-byte sums (from decide)
//   chunk_scan  — per chunk: inclusive prefix of new bytes within its block
//   flush       — one wave per range t walks the batch's blocks in order, finds flushes
//   place       — per chunk: container id / position; wave-cooperative copy into the arena;
//                 the designated chunk of each touched index entry writes its final value.
#include <cstdlib>

#include "launchers.hpp"

namespace hdrf {


__device__ __forceinline__ void range_bounds(int n, int t, int n_thread, int min_mt, int &c0, int &c1, int &nT)
{
    nT = n < min_mt ? 1 : n_thread;
    c0 = (int)((long long)n * t / nT);
    c1 = (int)((long long)n * (t + 1) / nT);
}

// ---- tile_scan: grid nblocks, 256 threads ------------------------------------------------
__global__ void __launch_bounds__(256) tile_scan_kernel(const BlockState *__restrict__ bst, int ntiles,
                                                        const uint32_t *__restrict__ tilesum,
                                                        uint32_t *__restrict__ tilepre, uint64_t *__restrict__ store_size,
                                                        int cap_blk)
{
    __shared__ uint32_t s[256];
    const int b = blockIdx.x;
    const int used = (bst[b].n_chunks + 255) / 256;
    uint32_t carry = 0;
    for (int base = 0; base < used; base += 256) {
        const int i = base + threadIdx.x;
        const uint32_t v = i < used ? tilesum[(size_t)b * ntiles + i] : 0u;
        s[threadIdx.x] = v;
        __syncthreads();
        for (int d = 1; d < 256; d <<= 1) {
            uint32_t t = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0u;
            __syncthreads();
            s[threadIdx.x] += t;
            __syncthreads();
        }
        if (i < used) tilepre[(size_t)b * ntiles + i] = carry + s[threadIdx.x] - v;
        carry += s[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) store_size[b] = carry;
}

// ---- chunk_scan: grid (ntiles, nblocks) --------------------------------------------------
__global__ void __launch_bounds__(256) chunk_scan_kernel(const BlockState *__restrict__ bst, int cap_blk, int ntiles,
                                                         const uint32_t *__restrict__ offsets,
                                                         const uint8_t *__restrict__ flags,
                                                         const uint32_t *__restrict__ tilepre, uint32_t *__restrict__ pre)
{
    __shared__ uint32_t s_w[4];
    const int b = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int n = bst[b].n_chunks;
    if (blockIdx.x * 256 >= n) return;
    const size_t c = (size_t)b * cap_blk + k;
    uint32_t v = 0;
    if (k < n && (flags[c] & 1)) {
        const uint32_t *off = offsets + (size_t)b * cap_blk;
        v = off[k] - (k ? off[k - 1] : 0u);
    }
    uint32_t incl = wave_incl_scan(v);
    if (lane_id() == 63) s_w[threadIdx.x >> 6] = incl;
    __syncthreads();
    const int wv = threadIdx.x >> 6;
    uint32_t add = tilepre[(size_t)b * ntiles + blockIdx.x];
    for (int i = 0; i < wv; i++) add += s_w[i];
    if (k < n) pre[c] = incl + add;
}

// first index c in [lo, hi) with pre[c] > thr (exists by construction); one wave, uniform
__device__ int wave_first_gt(const uint32_t *pre, int lo, int hi, uint64_t thr)
{
    const int l = lane_id();
    while (hi - lo > 64) {
        const int step = (hi - lo + 63) / 64;
        const int p = min(lo + (l + 1) * step - 1, hi - 1);
        const bool ok = (uint64_t)pre[p] > thr;
        const unsigned long long bal = ballot64(ok);
        const int j = __builtin_ctzll(bal);          // bal != 0: pre[hi-1] > thr
        const int nlo = lo + j * step;
        hi = min(lo + (j + 1) * step, hi);
        lo = nlo;
    }
    const bool ok = (lo + l < hi) && (uint64_t)pre[lo + l] > thr;
    const unsigned long long bal = ballot64(ok);
    return lo + __builtin_ctzll(bal);
}

// ---- flush: one workgroup, wave t handles range t ---------------------------------------
__global__ void __launch_bounds__(256) flush_kernel(StoreParams P, const BlockState *__restrict__ bst,
                                                    const uint64_t *__restrict__ store_size,
                                                    const uint32_t *__restrict__ pre, AllocState *__restrict__ alloc,
                                                    RangeState *__restrict__ rstate, FlushEv *__restrict__ events,
                                                    ClosedRec *__restrict__ closed, uint32_t *__restrict__ nclosed,
                                                    int *__restrict__ err)
{
    const int t = wave_id();
    if (t >= P.n_thread) return;
    const int l = lane_id();
    // per-lane prefetch of block-level quantities (lane = block, up to 64)
    int n_l = 0, c0_l = 0, c1_l = 0, act_l = 0;
    uint32_t base_l = 0, S_l = 0;
    if (l < P.nblocks) {
        n_l = bst[l].n_chunks;
        int nT;
        range_bounds(n_l, t, P.n_thread, P.min_mt, c0_l, c1_l, nT);
        act_l = (store_size[l] != 0 && t < nT) ? 1 : 0;
        const uint32_t *pb = pre + (size_t)l * P.cap_blk;
        base_l = c0_l > 0 ? pb[c0_l - 1] : 0u;
        S_l = (act_l && c1_l > c0_l) ? pb[c1_l - 1] - base_l : 0u;
    }
    uint32_t id = alloc->id[t], cur = alloc->cur[t], slot = alloc->slot[t], exists = alloc->exists[t];
    uint32_t pos = alloc->pos[t];
    int nev = 0;
    FlushEv *ev = events + (size_t)t * P.ev_cap;
    for (int b = 0; b < P.nblocks; b++) {
        const int act = rdlane(act_l, b);
        RangeState rs;
        rs.c_begin = (int)rdlane(c0_l, b);
        rs.c_end = (int)rdlane(c1_l, b);
        rs.base = rdlane(base_l, b);
        rs.active = act;
        rs.ev_begin = nev;
        rs.nflush = 0;
        rs.id0 = id; rs.slot0 = slot; rs.cur0 = cur;
        rs.total = 0;
        if (act) {
            if (!exists) { cur = 0; exists = 1; rs.cur0 = 0; }     // createNewFile (:726,736)
            const uint32_t S = rdlane(S_l, b);
            rs.total = S;
            int64_t cs = -(int64_t)cur;                              // container start, range-relative
            const uint32_t *pb = pre + (size_t)b * P.cap_blk;
            for (int guard = 0; (int64_t)S - cs > (int64_t)P.cmax; guard++) {
                if (guard > P.ev_cap) { if (l == 0) atomicOr(err, 8); break; }
                const uint64_t thr = (uint64_t)((int64_t)rs.base + cs + (int64_t)P.cmax);
                const int c = wave_first_gt(pb, rs.c_begin, rs.c_end, thr);
                const uint32_t X0 = (c > rs.c_begin ? pb[c - 1] : rs.base) - rs.base;
                if (l == 0) {
                    uint32_t ci = atomicAdd(nclosed, 1u);
                    if ((int)ci < P.closed_cap) {
                        ClosedRec cr; cr.id = id; cr.slot = slot; cr.len = (uint32_t)((int64_t)X0 - cs); cr.range = t;
                        closed[ci] = cr;
                    }
                }
                id = id + 1;
                // range t owns arena slots [t*per, (t+1)*per): a ring whose newest slot is its
                // open container, so recycling only ever overwrites t's oldest closed ones
                const uint32_t per = P.nslots / 4, base = (uint32_t)t * per;
                slot = base + (slot - base + 1) % per;
                cs = X0;
                if (nev < P.ev_cap) {
                    if (l == 0) { FlushEv e; e.chunk = c; e.new_id = id; e.new_slot = slot; e.base = X0; ev[nev] = e; }
                } else if (l == 0) atomicOr(err, 8);
                nev++;
                rs.nflush++;
            }
            cur = (uint32_t)((int64_t)S - cs);
            // the ring of range t must hold every container this batch closes plus the open one,
            // or a closed container's bytes would be overwritten before the host sees them
            if (nev >= (int)(P.nslots / 4) - 1 && l == 0) atomicOr(err, 32);
            pos = (uint32_t)((int64_t)S - (cs > 0 ? cs : 0));      // lastBlockID[t+4] (:808)
        }
        if (l == 0) rstate[(size_t)b * 4 + t] = rs;
    }
    if (l == 0) {
        alloc->id[t] = id; alloc->cur[t] = cur; alloc->slot[t] = slot; alloc->exists[t] = exists; alloc->pos[t] = pos;
    }
}

// ---- node-global allocator scan: the flush walk as a function of the incoming fill -------
// Range t's closes depend on the batch-start state only through the open container's fill x:
// the first close falls after the last chunk whose stream prefix is <= cmax - x, and from
// there on every close is fixed by the data.  fn_chain tabulates, for every distinct stream
// prefix v <= cmax (the possible first-close points), the final container start and the number
// of closes; the host (api.hip gx_apply_fn) evaluates the function for any x, so the ranks'
// allocator states come from one all-gather instead of a rank-to-rank chain.
// grid n_thread x 64: one wave per range, lane = block
__global__ void __launch_bounds__(64) fn_info_kernel(StoreParams P, const BlockState *__restrict__ bst,
                                                     const uint64_t *__restrict__ store_size,
                                                     const uint32_t *__restrict__ pre, FnBlock *__restrict__ fb,
                                                     FnRange *__restrict__ fr)
{
    __shared__ uint64_t sS[64];
    __shared__ uint32_t sN[64], sA[64];
    const int t = blockIdx.x, l = lane_id();
    FnBlock f{};
    if (l < P.nblocks) {
        const int n = bst[l].n_chunks;
        int c0, c1, nT;
        range_bounds(n, t, P.n_thread, P.min_mt, c0, c1, nT);
        f.act = (store_size[l] != 0 && t < nT) ? 1u : 0u;
        const uint32_t *pb = pre + (size_t)l * P.cap_blk;
        f.base = c0 > 0 ? pb[c0 - 1] : 0u;
        f.c0 = (uint32_t)c0;
        f.c1 = (uint32_t)c1;
        f.S = (f.act && c1 > c0) ? (uint64_t)(pb[c1 - 1] - f.base) : 0ull;
    }
    sS[l] = f.S;
    sN[l] = f.act ? f.c1 - f.c0 : 0u;
    sA[l] = f.act;
    __syncthreads();
    if (l == 0) {                                      // <= 64 blocks: serial exclusive offsets
        uint64_t off = 0;
        uint32_t coff = 0;
        FnRange r{};
        for (int b = 0; b < P.nblocks; b++) {
            const uint64_t Sb = sS[b];
            const uint32_t nb = sN[b];
            if (sA[b]) { r.any = 1; r.base_last = off; r.S_last = Sb; }
            sS[b] = off;
            sN[b] = coff;
            off += Sb;
            coff += nb;
        }
        r.S = off;
        r.nstream = coff;
        fr[t] = r;
    }
    __syncthreads();
    if (l < P.nblocks) {
        f.off = sS[l];
        f.coff = sN[l];
        fb[(size_t)t * 64 + l] = f;
    }
}

// grid (ceil((max stream chunks + 1) / 256), n_thread) x 256: candidate i of range t is the
// stream prefix v_i before stream chunk i (v_0 = 0).  Candidates with v_i <= cmax whose chunk
// i - 1 added bytes (the distinct prefixes) run the close chain from a container starting at
// v_i; out[i] = {v_i, final container start, closes | repeat flag}; K[t] = candidates with
// v_i <= cmax (a prefix, v is nondecreasing).
__global__ void __launch_bounds__(256) fn_chain_kernel(StoreParams P, const uint32_t *__restrict__ pre,
                                                       const FnBlock *__restrict__ fb, const FnRange *__restrict__ fr,
                                                       uint64_t *__restrict__ out, int64_t kcap,
                                                       unsigned long long *__restrict__ K, int *__restrict__ err)
{
    __shared__ FnBlock sb[64];
    const int t = blockIdx.y;
    const int nb = P.nblocks;
    if ((int)threadIdx.x < nb) sb[threadIdx.x] = fb[(size_t)t * 64 + threadIdx.x];
    __syncthreads();
    const FnRange R = fr[t];
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i > (int64_t)R.nstream) return;
    // stream chunk j = i - 1 -> (block, chunk); v_i = prefix after it, w = prefix before it
    uint64_t v = 0, w = 0;
    if (i > 0) {
        const uint32_t j = (uint32_t)(i - 1);
        int b = 0;
        for (int q = 0; q < nb; q++)
            if (sb[q].act && sb[q].c1 > sb[q].c0 && sb[q].coff <= j) b = q;
        const uint32_t *pb = pre + (size_t)b * P.cap_blk;
        const uint32_t c = sb[b].c0 + (j - sb[b].coff);
        v = sb[b].off + (uint64_t)(pb[c] - sb[b].base);
        w = sb[b].off + (c > sb[b].c0 ? (uint64_t)(pb[c - 1] - sb[b].base) : 0ull);
    }
    if (v > (uint64_t)P.cmax) return;
    if (i >= kcap) { atomicOr(err, 1024); return; }
    atomicMax(K + t, (unsigned long long)(i + 1));
    uint64_t *o = out + ((size_t)t * kcap + i) * 3;
    o[0] = v;
    if (i > 0 && v == w) { o[1] = 0; o[2] = 1ull << 63; return; }   // same prefix as candidate i - 1
    int64_t cs = (int64_t)v;
    uint64_t n = 0;
    while ((int64_t)R.S - cs > (int64_t)P.cmax) {
        const int64_t thr = cs + (int64_t)P.cmax;
        int b = -1;                                    // first active block ending past thr
        for (int q = 0; q < nb && b < 0; q++)
            if (sb[q].act && (int64_t)(sb[q].off + sb[q].S) > thr) b = q;
        if (b < 0 || n > (uint64_t)P.ev_cap * 64) { atomicOr(err, 1024); return; }
        const uint32_t *pb = pre + (size_t)b * P.cap_blk;
        const uint64_t lim = (uint64_t)(thr - (int64_t)sb[b].off) + sb[b].base;   // first pb[c] > lim
        uint32_t lo = sb[b].c0, hi = sb[b].c1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((uint64_t)pb[mid] > lim) hi = mid; else lo = mid + 1;
        }
        cs = (int64_t)sb[b].off + (lo > sb[b].c0 ? (int64_t)(pb[lo - 1] - sb[b].base) : 0);
        n++;
    }
    o[1] = (uint64_t)cs;
    o[2] = n;
}

// ---- the flush function as a fixed-size descriptor (node-global allocator scan on the device) ----
// fn_chain leaves K[t] candidate rows per range, rows that repeat the previous prefix flagged; the
// distinct prefixes v <= cmax are at most cmax / (window + 2) + nblocks + 1 (every chunk is >= window
// + 2 bytes except a block's last), so the packed descriptor has a fixed size and ranks exchange it
// with one all-gather of equal parts.  grid n_thread x 256
uint64_t gx_fn_mcap(uint32_t cmax, int window, int max_batch)
{
    return (uint64_t)cmax / (uint64_t)(window + 2) + (uint64_t)max_batch + 2;
}
uint64_t gx_fn_bytes(uint32_t cmax, int window, int max_batch)
{
    return (sizeof(GxFnHead) + 3 * gx_fn_mcap(cmax, window, max_batch) * sizeof(GxFnRow) + 255) & ~(uint64_t)255;   // <= 3 ranges
}

__global__ void __launch_bounds__(256) fn_pack_kernel(int n_thread, const FnRange *__restrict__ fr,
                                                      const uint64_t *__restrict__ rows, int64_t kcap,
                                                      const unsigned long long *__restrict__ K, uint64_t mcap,
                                                      uint8_t *__restrict__ desc, int *__restrict__ err)
{
    __shared__ uint32_t s_w[4];
    const int t = blockIdx.x, tid = threadIdx.x;
    GxFnHead *h = (GxFnHead *)desc;
    GxFnRow *out = (GxFnRow *)(desc + sizeof(GxFnHead)) + (size_t)t * mcap;
    const FnRange R = fr[t];
    const uint64_t k = K[t];
    uint32_t m = 0;
    for (uint64_t base = 0; base < k; base += 256) {
        const uint64_t i = base + tid;
        const uint64_t *r = rows + ((size_t)t * kcap + i) * 3;
        const bool keep = i < k && !(r[2] >> 63);
        const uint32_t incl = wave_incl_scan(keep ? 1u : 0u);
        if (lane_id() == 63) s_w[tid >> 6] = incl;
        __syncthreads();
        uint32_t off = m;
        for (int w = 0; w < (tid >> 6); w++) off += s_w[w];
        const uint32_t tot = s_w[0] + s_w[1] + s_w[2] + s_w[3];
        if (keep) {
            const uint64_t j = off + incl - 1;
            if (j < mcap) {
                GxFnRow row;
                row.v = (uint32_t)r[0];
                row.cur = (uint32_t)(R.S - r[1]);               // S - cs <= cmax
                row.n = (uint32_t)r[2];
                row.pad = 0;
                out[j] = row;
            } else {
                atomicOr(err, 1024);
            }
        }
        m += tot;
        __syncthreads();
    }
    if (tid == 0) {
        if (t == 0) { h->n_thread = (uint64_t)n_thread; h->mcap = mcap; }
        h->any[t] = R.any; h->S[t] = R.S; h->base_last[t] = R.base_last; h->S_last[t] = R.S_last;
        h->m[t] = m;
        if (R.any && (m == 0 || out[0].v != 0)) atomicOr(err, 1024);   // the first candidate is v = 0
    }
}

hipError_t launch_fn_pack(int n_thread, const FnRange *fr, const uint64_t *rows, int64_t kcap,
                          const unsigned long long *K, uint64_t mcap, void *desc, int *err, hipStream_t st)
{
    hipLaunchKernelGGL(fn_pack_kernel, dim3(n_thread), dim3(256), 0, st, n_thread, fr, rows, kcap, K, mcap,
                       (uint8_t *)desc, err);
    return hipGetLastError();
}

// The node's allocator through every rank's flush function, rank order (api.hip gx_apply_fn on the
// device): lane t < n_thread evaluates range t, the ranges are independent.  One wave.
__global__ void __launch_bounds__(64) gx_scan_kernel(const uint8_t *__restrict__ descs, uint64_t fn_bytes, int G,
                                                     int rank, int n_thread, uint32_t per, uint32_t cmax,
                                                     AllocState *__restrict__ alloc, AllocState *__restrict__ states,
                                                     int *__restrict__ err)
{
    const int t = lane_id();
    __shared__ AllocState sA;
    if (t == 0) sA = *alloc;
    __syncthreads();
    for (int r = 0; r < G; r++) {
        if (r == rank && t == 0) states[0] = sA;
        __syncthreads();
        const GxFnHead *h = (const GxFnHead *)(descs + (size_t)r * fn_bytes);
        const GxFnRow *rows = (const GxFnRow *)(descs + (size_t)r * fn_bytes + sizeof(GxFnHead));
        if (t == 0 && (h->n_thread != (uint64_t)n_thread || sizeof(GxFnHead) + 3 * h->mcap * sizeof(GxFnRow) > fn_bytes))
            atomicOr(err, 512);
        if (t < n_thread && h->n_thread == (uint64_t)n_thread && h->any[t]) {
            const uint64_t m = h->m[t], S = h->S[t];
            const GxFnRow *v = rows + (size_t)t * h->mcap;
            const int64_t x = sA.exists[t] ? (int64_t)sA.cur[t] : 0;
            int64_t cs = -x, n = 0;
            uint32_t cur = (uint32_t)((int64_t)S + x);
            if (x + (int64_t)S > (int64_t)cmax) {
                if (m == 0 || m > h->mcap) {
                    atomicOr(err, 512);
                } else {
                    const uint64_t thr = (uint64_t)((int64_t)cmax - x);   // largest v <= thr (v_0 = 0)
                    uint64_t lo = 0, hi = m;
                    while (hi - lo > 1) {
                        const uint64_t mid = (lo + hi) >> 1;
                        if ((uint64_t)v[mid].v <= thr) lo = mid; else hi = mid;
                    }
                    cur = v[lo].cur;
                    cs = (int64_t)S - (int64_t)cur;
                    n = 1 + (int64_t)v[lo].n;
                }
            }
            const uint32_t base = (uint32_t)t * per;
            sA.id[t] += (uint32_t)n;
            sA.slot[t] = base + (uint32_t)(((int64_t)(sA.slot[t] - base) + n) % per);
            sA.cur[t] = cur;
            sA.exists[t] = 1;
            const int64_t bl = (int64_t)h->base_last[t];
            sA.pos[t] = (uint32_t)((int64_t)h->S_last[t] - (cs - bl > 0 ? cs - bl : 0));
        }
        __syncthreads();
        if (r == rank && t == 0) states[1] = sA;
        __syncthreads();
    }
    if (t == 0) {
        states[2] = sA;
        *alloc = states[0];                                  // the flush walk starts from this rank's state
    }
}

hipError_t launch_gx_scan(const void *descs, uint64_t fn_bytes, int G, int rank, int n_thread, uint32_t per,
                          uint32_t cmax, AllocState *alloc, AllocState *states, int *err, hipStream_t st)
{
    hipLaunchKernelGGL(gx_scan_kernel, dim3(1), dim3(64), 0, st, (const uint8_t *)descs, fn_bytes, G, rank, n_thread,
                       per, cmax, alloc, states, err);
    return hipGetLastError();
}

// workgroup-cooperative copy of one contiguous run (16-B aligned destination stores)
template <bool NT>
__device__ __forceinline__ void wg_copy(uint8_t *dst, const uint8_t *src, uint32_t len, bool deep = false)
{
    const int t = threadIdx.x;
    uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
    if (head > len) head = len;
    if ((uint32_t)t < head) dst[t] = src[t];
    uint8_t *d = dst + head;
    const uint8_t *sp = src + head;
    const uint32_t n16 = (len - head) >> 4;
    const int sh = (int)((uintptr_t)sp & 15);
    const uint8_t *sa = sp - sh;
    uint32_t i = t;
    if (deep)                                       // (uniform) four 16-B words per thread in flight
        for (; i + 768 < n16; i += 1024) {
            const uint4 v0 = load16_shift<NT>(sa + 16 * (size_t)i, sh);
            const uint4 v1 = load16_shift<NT>(sa + 16 * (size_t)(i + 256), sh);
            const uint4 v2 = load16_shift<NT>(sa + 16 * (size_t)(i + 512), sh);
            const uint4 v3 = load16_shift<NT>(sa + 16 * (size_t)(i + 768), sh);
            st16_t<NT>(d + 16 * (size_t)i, v0);
            st16_t<NT>(d + 16 * (size_t)(i + 256), v1);
            st16_t<NT>(d + 16 * (size_t)(i + 512), v2);
            st16_t<NT>(d + 16 * (size_t)(i + 768), v3);
        }
    for (; i + 256 < n16; i += 512) {               // two 16-B words per thread in flight
        const uint4 v0 = load16_shift<NT>(sa + 16 * (size_t)i, sh);
        const uint4 v1 = load16_shift<NT>(sa + 16 * (size_t)(i + 256), sh);
        st16_t<NT>(d + 16 * (size_t)i, v0);
        st16_t<NT>(d + 16 * (size_t)(i + 256), v1);
    }
    for (; i < n16; i += 256) st16_t<NT>(d + 16 * (size_t)i, load16_shift<NT>(sa + 16 * (size_t)i, sh));
    const uint32_t tb = head + 16 * n16;
    if ((uint32_t)t < len - tb) dst[tb + t] = src[tb + t];
}

// ---- place: grid (ntiles, nblocks) ------------------------------------------------------
template <bool NT>
__global__ void __launch_bounds__(256) place_kernel(StoreParams P, const BlockDesc *__restrict__ blocks,
                                                    const BlockState *__restrict__ bst,
                                                    const uint32_t *__restrict__ offsets,
                                                    const uint8_t *__restrict__ flags, const uint32_t *__restrict__ pre,
                                                    const RangeState *__restrict__ rstate,
                                                    const FlushEv *__restrict__ events, const uint32_t *__restrict__ slot,
                                                    IndexEntry *__restrict__ tab, uint8_t *__restrict__ arena,
                                                    uint32_t *__restrict__ place_cid, uint32_t *__restrict__ place_pos,
                                                    GxPlace gx, int prio, const uint8_t *__restrict__ dcnt)
{
    if (prio) __builtin_amdgcn_s_setprio(2);        // HDRF_SETPRIO bit 5
    const int b = blockIdx.y;
    const int k = blockIdx.x * 256 + threadIdx.x;
    const int n = bst[b].n_chunks;
    if (blockIdx.x * 256 >= n) return;
    const BlockDesc bd = blocks[b];
    const size_t c = (size_t)b * P.cap_blk + k;
    const uint32_t *off = offsets + (size_t)b * P.cap_blk;
    uint8_t f = 0;
    uint32_t start = 0, len = 0, cid = 0, pos = 0, aslot = 0, x3_ri = 0;
    bool do_copy = false, x3_want = false;
    if (k < n) {
        f = flags[c];
        start = k ? off[k - 1] : 0u;
        len = off[k] - start;
        if (f & 1) {
            int c0, c1, nT, t = 0;
            for (int tt = 0; tt < 3; tt++) {
                range_bounds(n, tt, P.n_thread, P.min_mt, c0, c1, nT);
                if (tt < nT && k >= c0 && k < c1) { t = tt; break; }
            }
            const RangeState rs = rstate[(size_t)b * 4 + t];
            if (rs.active) {
                const uint32_t X0 = pre[c] - len - rs.base;
                cid = rs.id0; aslot = rs.slot0;
                int64_t cs = -(int64_t)rs.cur0;
                const FlushEv *ev = events + (size_t)t * P.ev_cap + rs.ev_begin;
                for (int i = 0; i < rs.nflush; i++) {      // few events per (block, range)
                    const FlushEv e = ev[i];
                    if (e.chunk > k) break;
                    cid = e.new_id; aslot = e.new_slot; cs = e.base;
                }
                pos = (uint32_t)((int64_t)X0 - cs);
                do_copy = len > 0;
            }
            if (gx.part != 2) {
                place_cid[c] = cid;
                place_pos[c] = pos;
            }
        }
        if (gx.part != 2) {                                // (the copy part: part 1 wrote the index)
        bool desig = (f & 2) != 0;                         // in the entry's min block ...
        IndexEntry *e = tab + slot[c];
        if (dcnt) desig = (f & 32) != 0;                   // (idx_finalize already decided and cleared)
        else if (desig && (f & 16))                        // ... and its last occurrence there
            desig = (uint32_t)e->first == (uint32_t)(k + 1);
        if (desig && gx.x3) {                              // node-global index (gx.hip): the
            if (f & 4) {                                   // owner commits the new entry's location
                x3_ri = e->cid;                            // (its X3 record, written below)
                x3_want = true;
            }
        } else if (desig) {                                // designated: final index value
            const uint32_t cnt = dcnt ? (uint32_t)dcnt[c] : (uint32_t)__popcll(e->mask);
            if (f & 4) {
                set_ncopy(e, cnt);
                e->cid = cid; e->start = pos; e->stop = pos + ((f & 1) && do_copy ? len : 0u);
            } else {
                set_ncopy(e, e->ncopy + cnt);
            }
            if (!dcnt) {
                e->mask = 0;
                e->first = 0;
            }
        }
        }
    }
    // the runs' LDS (below); the X3 reservation borrows s_cid / s_pend, so the kernel keeps its
    // single-node LDS size: its own 768 B (7952 instead of 7184 B per workgroup) shifted the config-2
    // balance between the place copy and the chunking chain (B2 3.6 -> 3.9 ms per batch) and cost
    // 4.7 % (1103 vs 1054 GB/s, three A/B pairs, profiles/r06_placelds_ab.txt)
    __shared__ uint32_t s_cid[256], s_flag[256];
    __shared__ __attribute__((aligned(8))) uint32_t s_pend[256];
    __shared__ uint32_t r_src[256], r_end[256], r_dst_lo[256], r_dst_hi[256];
    __shared__ uint32_t s_wsum[4];
    if (gx.x3 && gx.part != 2) {                          // (uniform) the X3 location records, one
        const int d = (int)(x3_ri / (uint64_t)gx.cap);     // global atomic per (workgroup, owner): one per
        const unsigned long long i =                       // record serialised at the memory side (gx.hip)
            wg_reserve(gx.counts, x3_want ? d : 0, x3_want, gx.G, s_cid, (unsigned long long *)s_pend);
        if (x3_want) {
            uint32_t *rec = gx.x3 + ((size_t)d * gx.cap + i) * 4;
            rec[0] = gx.x2[2 * (size_t)x3_ri];
            rec[1] = cid; rec[2] = pos; rec[3] = pos + ((f & 1) && do_copy ? len : 0u);
        }
        __syncthreads();                                   // (s_cid / s_pend are rewritten below)
    }
    if (gx.part == 1) return;                              // placement part: no arena copy
    // ---- runs: consecutive new chunks of this tile that are contiguous in one container are
    //      one contiguous source span and one contiguous destination span -> one copy each
    const int tid = threadIdx.x;
    s_cid[tid] = do_copy ? cid : 0xffffffffu;
    s_pend[tid] = pos + len;
    __syncthreads();
    const bool cont = do_copy && tid > 0 && s_cid[tid - 1] == cid && s_pend[tid - 1] == pos;
    const bool rstart = do_copy && !cont;
    s_flag[tid] = cont ? 1u : 0u;
    // exclusive scan of run starts (wave scan + cross-wave sums)
    const uint32_t incl = wave_incl_scan(rstart ? 1u : 0u);
    if (lane_id() == 63) s_wsum[tid >> 6] = incl;
    __syncthreads();
    uint32_t base_idx = 0;
    for (int i = 0; i < (tid >> 6); i++) base_idx += s_wsum[i];
    const uint32_t nruns = s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
    const uint32_t ridx = base_idx + incl - (rstart ? 1u : 0u);
    if (rstart) {
        const uint64_t dsto = (uint64_t)aslot * P.cmax + pos;
        r_src[ridx] = start;
        r_dst_lo[ridx] = (uint32_t)dsto;
        r_dst_hi[ridx] = (uint32_t)(dsto >> 32);
    }
    const bool last = do_copy && !(tid + 1 < 256 && s_flag[tid + 1]);
    if (last) r_end[base_idx + incl - 1] = start + len;       // run index of this (continuing) run
    __syncthreads();
    for (uint32_t r = 0; r < nruns; r++) {
        const uint64_t dsto = ((uint64_t)r_dst_hi[r] << 32) | r_dst_lo[r];
        wg_copy<NT>(arena + dsto, bd.data + r_src[r], r_end[r] - r_src[r], P.place_deep != 0);
    }
}

int stream_knobs()
{
    // r02 A/B on the config-2 bench (scripts/ab_nt.txt): 973 / 984 GB/s off, 994 / 995 with both
    static const int k = [] { const char *e = getenv("HDRF_NT"); return e ? atoi(e) : 3; }();
    return k;
}

hipError_t launch_store_scan(const StoreParams &P, const BlockState *bst, const uint32_t *offsets, const uint8_t *flags,
                             const uint32_t *tilesum, uint32_t *tilepre, uint64_t *store_size, uint32_t *pre,
                             hipStream_t st)
{
    hipLaunchKernelGGL(tile_scan_kernel, dim3(P.nblocks), dim3(256), 0, st, bst, P.ntiles, tilesum, tilepre,
                       store_size, P.cap_blk);
    hipLaunchKernelGGL(chunk_scan_kernel, dim3(P.ntiles, P.nblocks), dim3(256), 0, st, bst, P.cap_blk, P.ntiles,
                       offsets, flags, tilepre, pre);
    return hipGetLastError();
}

hipError_t launch_store_flush(const StoreParams &P, const BlockState *bst, const uint64_t *store_size, const uint32_t *pre,
                              AllocState *alloc, RangeState *rstate, FlushEv *events, ClosedRec *closed,
                              uint32_t *nclosed, int *err, hipStream_t st)
{
    hipLaunchKernelGGL(flush_kernel, dim3(1), dim3(256), 0, st, P, bst, store_size, pre, alloc, rstate, events, closed,
                       nclosed, err);
    return hipGetLastError();
}

hipError_t launch_flush_fn(const StoreParams &P, const BlockState *bst, const uint64_t *store_size, const uint32_t *pre,
                           FnBlock *fb, FnRange *fr, uint64_t *out, int64_t kcap, unsigned long long *K, int *err,
                           hipStream_t st)
{
    hipLaunchKernelGGL(fn_info_kernel, dim3(P.n_thread), dim3(64), 0, st, P, bst, store_size, pre, fb, fr);
    const int64_t nmax = (int64_t)P.nblocks * P.cap_blk + 1;
    hipLaunchKernelGGL(fn_chain_kernel, dim3((unsigned)((nmax + 255) / 256), P.n_thread), dim3(256), 0, st, P, pre, fb, fr,
                       out, kcap, K, err);
    return hipGetLastError();
}

hipError_t launch_store_place(const StoreParams &P, const BlockDesc *d_blocks, const BlockState *bst,
                              const uint32_t *offsets, const uint8_t *flags, const uint32_t *pre,
                              const RangeState *rstate, const FlushEv *events, const uint32_t *slot, IndexEntry *tab,
                              uint8_t *arena, uint32_t *place_cid, uint32_t *place_pos, const GxPlace &gx,
                              hipStream_t st, const uint8_t *dcnt)
{
    if (gx.x3 && gx.part != 2)
        if (hipError_t e = hipMemsetAsync(gx.counts, 0, sizeof(unsigned long long) * gx.G, st)) return e;
    if (stream_knobs() & 2)
        hipLaunchKernelGGL(place_kernel<true>, dim3(P.ntiles, P.nblocks), dim3(256), P.place_lds, st, P, d_blocks, bst,
                           offsets, flags, pre, rstate, events, slot, tab, arena, place_cid, place_pos, gx,
                           (setprio_mask() >> 5) & 1, dcnt);
    else
        hipLaunchKernelGGL(place_kernel<false>, dim3(P.ntiles, P.nblocks), dim3(256), P.place_lds, st, P, d_blocks, bst,
                           offsets, flags, pre, rstate, events, slot, tab, arena, place_cid, place_pos, gx,
                           (setprio_mask() >> 5) & 1, dcnt);
    return hipGetLastError();
}

hipError_t launch_store(const StoreParams &P, const BlockDesc *d_blocks, const BlockState *bst,
                        const uint32_t *offsets, const uint8_t *flags, const uint32_t *tilesum, uint32_t *tilepre,
                        uint64_t *store_size, uint32_t *pre, AllocState *alloc, RangeState *rstate, FlushEv *events,
                        ClosedRec *closed, uint32_t *nclosed, const uint32_t *slot, IndexEntry *tab, uint8_t *arena,
                        uint32_t *place_cid, uint32_t *place_pos, int *err, hipStream_t st, Marker *mk,
                        const GxPlace *gx, const uint8_t *dcnt)
{
    const GxPlace gxp = gx ? *gx : GxPlace{};
    mk->mark(st);
    hipError_t e = launch_store_scan(P, bst, offsets, flags, tilesum, tilepre, store_size, pre, st);
    mk->mark(st);
    if (e == hipSuccess) e = launch_store_flush(P, bst, store_size, pre, alloc, rstate, events, closed, nclosed, err, st);
    mk->mark(st);
    if (e == hipSuccess)
        e = launch_store_place(P, d_blocks, bst, offsets, flags, pre, rstate, events, slot, tab, arena, place_cid,
                               place_pos, gxp, st, dcnt);
    mk->mark(st);
    mk->mark(st);   // spare stage (kept so stage indices stay stable)
    return e;
}

// storeDB's recipe SET (DN/DataDeduplicator.java:372-392): copy each block's digests (already
// contiguous in the batch slot) into the device recipe store; grid (n, kRecipeWgs) x 256, 16 B per
// lane per step (4-B aligned dwordx4: the digest rows and the store's records are 4-B aligned).  The
// copy runs on stream C beside the pipeline: with one dword per lane and 8 workgroups per block it held
// 256 workgroups for ~540 us per batch (profiles/r06_c2_kernel_stats.csv).
typedef uint32_t u32x4r __attribute__((ext_vector_type(4), aligned(4)));
constexpr int kRecipeWgs = 32;
__global__ void __launch_bounds__(256) recipe_copy_kernel(const RecipeCopy *__restrict__ jobs, int n)
{
    if ((int)blockIdx.x >= n) return;
    const RecipeCopy j = jobs[blockIdx.x];
    const uint32_t *src = (const uint32_t *)(uintptr_t)j.src;
    uint32_t *dst = (uint32_t *)(uintptr_t)j.dst;
    const uint32_t nq = j.words >> 2, stride = gridDim.y * 256;
    for (uint32_t i = blockIdx.y * 256 + threadIdx.x; i < nq; i += stride)
        *(u32x4r *)(dst + 4 * i) = *(const u32x4r *)(src + 4 * i);
    const uint32_t t = 4 * nq + blockIdx.y * 256 + threadIdx.x;     // the last words (< 4)
    if (t < j.words && blockIdx.y * 256 + threadIdx.x < 4) dst[t] = src[t];
}

// Container drain (api.hip hdrf_drain_containers) into pinned host memory: the CUs write the bytes
// straight across PCIe (the host buffer is device-mapped), so the D2H of a DataNode's container files
// runs beside the SDMA engine's H2D copies of the next blocks instead of queueing behind them.
// Items (job j, piece y of kXferPiece bytes), numbered y * jobs + j; `wgs` workgroups loop over them
// (0: one workgroup per item).  The drain shares the link with the next blocks' H2D copies: a full
// grid's flood of writes cuts the copies under it from 55.7 to 44.6 GB/s (config 5 trace, r04); five
// workgroups drain about as fast and leave the copies at 54.9 GB/s.
constexpr uint64_t kXferPiece = 256 << 10;
__global__ void __launch_bounds__(256) xfer_kernel(const XferJob *__restrict__ jobs, int njobs, uint32_t pieces)
{
    const uint64_t total = (uint64_t)njobs * pieces, step = (uint64_t)gridDim.x * gridDim.y;
    for (uint64_t it = blockIdx.x + (uint64_t)blockIdx.y * gridDim.x; it < total; it += step) {
        const XferJob J = jobs[it % (uint64_t)njobs];
        const uint64_t o = (it / (uint64_t)njobs) * kXferPiece;
        if (o >= J.n) continue;
        const uint64_t n = J.n - o < kXferPiece ? J.n - o : kXferPiece;
        wg_copy<false>((uint8_t *)(uintptr_t)(J.dst + o), (const uint8_t *)(uintptr_t)(J.src + o), (uint32_t)n);
    }
}

hipError_t launch_xfer(const XferJob *jobs, int n, uint64_t max_bytes, int wgs, hipStream_t st)
{
    const uint64_t pieces = (max_bytes + kXferPiece - 1) / kXferPiece;
    if (n <= 0 || pieces == 0) return hipGetLastError();
    if (wgs > 0)
        hipLaunchKernelGGL(xfer_kernel, dim3((unsigned)wgs), dim3(256), 0, st, jobs, n, (uint32_t)pieces);
    else
        hipLaunchKernelGGL(xfer_kernel, dim3(n, (unsigned)pieces), dim3(256), 0, st, jobs, n, (uint32_t)pieces);
    return hipGetLastError();
}

hipError_t launch_recipe_copy(const RecipeCopy *jobs, int n, hipStream_t st)
{
    if (n > 0) hipLaunchKernelGGL(recipe_copy_kernel, dim3(n, kRecipeWgs), dim3(256), 0, st, jobs, n);
    return hipGetLastError();
}

}  // namespace hdrf
