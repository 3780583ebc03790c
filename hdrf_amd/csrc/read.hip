// read.hip — block reconstruction (the read side) on gfx950.
//
// Reference: DataConstructor(blkID, recipe) -> quickBuildMT, DN/DataConstructor.java:73-250,
// 360-417: the recipe [BE32 size | digest_0 .. digest_{n-1}] is split into digests
// (:221-230), every digest is looked up in Redis (pipelined GET, :368-371), chunkMeta.process
// assigns each chunk its block offset as the running sum of the decoded lengths (:375-377,
// DN/chunkMeta.java:35-60), and threadedConstructor copies container[start, stop) to
// data[bbStart, bbStop) (:474-531).
//
//   rd_lookup — one lane per chunk: probe the index (same open addressing as index.hip), decode
//               (container id, start, stop), and the readable copy of the container (an arena
//               slot, or a container loaded back from its file with hdrf_container_load)
//   rd_scan   — one workgroup: exclusive prefix of the chunk lengths (block offsets) + total
//   rd_gather — one wave per chunk: 16-B-per-lane copy arena -> output block
//   gx_locate — node-global contexts: the owner's lookup of the digests it owns (location +
//               placing rank); each rank then gathers the chunks it placed (hdrf_gx_read_*)
#include "launchers.hpp"

namespace hdrf {

struct RdChunk {
    uint32_t slot;       // index of the container in the readable list (0xffffffff: missing)
    uint32_t start, len;
    uint32_t off;        // offset in the rebuilt block
};

// probe the index for one digest (the open addressing of index.hip); nullptr when absent
template <int HW>
__device__ const IndexEntry *rd_probe(const uint32_t *dw, const IndexEntry *__restrict__ tab, int log2cap,
                                      unsigned long long key)
{
    const unsigned long long tag = tag_word(dw, key);
    const uint64_t mask = (1ull << log2cap) - 1;
    uint64_t h = tag_home(tag, log2cap);
    for (uint64_t probe = 0; probe <= mask; probe++) {
        const IndexEntry &e = tab[h];
        if (!tag_live(e.tag, key)) return nullptr;           // empty (or of an older epoch)
        if (e.tag == tag && entry_matches<HW>(e, dw)) return &e;
        h = (h + 1) & mask;
    }
    return nullptr;
}

template <int HW>
__global__ void __launch_bounds__(256) rd_lookup_kernel(const uint32_t *__restrict__ dig, int n,
                                                        const IndexEntry *__restrict__ tab, int log2cap,
                                                        unsigned long long tag_mask, const uint32_t *__restrict__ cids,
                                                        int ncont, RdChunk *__restrict__ out, int *__restrict__ err)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    uint32_t dw[HW];
#pragma unroll
    for (int i = 0; i < HW; i++) dw[i] = dig[(size_t)k * HW + i];
    RdChunk r;
    r.slot = 0xffffffffu; r.start = 0; r.len = 0; r.off = 0;
    const IndexEntry *e = rd_probe<HW>(dw, tab, log2cap, tag_mask);
    if (e) {
        r.start = e->start;
        r.len = e->stop - e->start;                    // chunkMeta.length = blockStop - blockStart
        int lo = 0, hi = ncont;                        // readable container list, sorted by id
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (cids[mid] < e->cid) lo = mid + 1; else hi = mid;
        }
        if (lo < ncont && cids[lo] == e->cid) r.slot = (uint32_t)lo;
    }
    if (!e || (r.slot == 0xffffffffu && r.len != 0)) atomicOr(err, 1);   // empty chunks need no container
    out[k] = r;
}

// Node-global read (G > 1): the owner's lookup of the recipe digests it owns (first digest word
// mod G == rank).  loc[k] = {container id, start, stop, placing rank + 1} for an owned digest,
// zeros for the others; an owned digest that is absent sets *err.  The placing rank is the X3
// source own_commit_kernel recorded in bits 24-31 of the entry's container id.
template <int HW>
__global__ void __launch_bounds__(256) gx_locate_kernel(const uint32_t *__restrict__ dig, int n,
                                                        const IndexEntry *__restrict__ tab, int log2cap,
                                                        unsigned long long tag_mask, int G, int rank,
                                                        uint32_t *__restrict__ loc, int *__restrict__ err)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n) return;
    uint32_t dw[HW];
#pragma unroll
    for (int i = 0; i < HW; i++) dw[i] = dig[(size_t)k * HW + i];
    uint4 v = make_uint4(0, 0, 0, 0);
    if ((int)(dw[0] % (uint32_t)G) == rank) {
        const IndexEntry *e = rd_probe<HW>(dw, tab, log2cap, tag_mask);
        if (e) v = make_uint4(e->cid & 0xffffffu, e->start, e->stop, e->cid >> 24);
        if (!e || v.w == 0u) atomicOr(err, 1);        // missing, or a location without its placer
    }
    *(uint4 *)(loc + 4 * (size_t)k) = v;
}

// one workgroup of 1024 threads: off[k] = sum of len[0..k), total -> *total
__global__ void __launch_bounds__(1024) rd_scan_kernel(RdChunk *__restrict__ c, int n, uint64_t *__restrict__ total)
{
    __shared__ uint32_t s_w[16];
    __shared__ uint64_t s_carry;
    const int t = threadIdx.x;
    if (t == 0) s_carry = 0;
    __syncthreads();
    for (int base = 0; base < n; base += 1024) {
        const int k = base + t;
        const uint32_t v = k < n ? c[k].len : 0u;
        const uint32_t incl = wave_incl_scan(v);
        if (lane_id() == 63) s_w[t >> 6] = incl;
        __syncthreads();
        uint32_t add = 0, tot = 0;
        for (int i = 0; i < 16; i++) {
            if (i < (t >> 6)) add += s_w[i];
            tot += s_w[i];
        }
        const uint64_t carry = s_carry;
        if (k < n) c[k].off = (uint32_t)(carry + add + incl - v);
        __syncthreads();
        if (t == 0) s_carry = carry + tot;
        __syncthreads();
    }
    if (t == 0) *total = s_carry;
}

// grid ceil(n/4) x 256: wave w of the workgroup copies chunk 4*blockIdx.x + w
__global__ void __launch_bounds__(256) rd_gather_kernel(const RdChunk *__restrict__ c, int n,
                                                        const uint64_t *__restrict__ bases, uint8_t *__restrict__ out)
{
    const int k = blockIdx.x * 4 + wave_id();
    if (k >= n) return;
    const RdChunk r = c[k];
    if (r.slot == 0xffffffffu) return;
    const uint8_t *src = (const uint8_t *)(uintptr_t)bases[r.slot] + r.start;
    uint8_t *dst = out + r.off;
    const int l = lane_id();
    const uint32_t len = r.len;
    uint32_t head = (uint32_t)((16 - ((uintptr_t)dst & 15)) & 15);
    if (head > len) head = len;
    if ((uint32_t)l < head) dst[l] = src[l];
    uint8_t *d = dst + head;
    const uint8_t *sp = src + head;
    const uint32_t n16 = (len - head) >> 4;
    const int sh = (int)((uintptr_t)sp & 15);
    const uint8_t *sa = sp - sh;
    for (uint32_t i = l; i < n16; i += 64) st16(d + 16 * (size_t)i, load16_shift(sa + 16 * (size_t)i, sh));
    const uint32_t tb = head + 16 * n16;
    for (uint32_t i = tb + l; i < len; i += 64) dst[i] = src[i];
}

hipError_t launch_reconstruct(int hasher, const uint32_t *dig, int n, const IndexEntry *tab, int log2cap,
                              unsigned long long tag_mask, const uint32_t *cids, const uint64_t *bases, int ncont,
                              void *chunks, uint64_t *total, uint8_t *out, int *err, hipStream_t st, bool gather)
{
    RdChunk *c = (RdChunk *)chunks;
    if (n <= 0) return hipSuccess;
    if (!gather) {
        const dim3 g((n + 255) / 256);
        if (hasher == 0)
            hipLaunchKernelGGL(rd_lookup_kernel<5>, g, dim3(256), 0, st, dig, n, tab, log2cap, tag_mask, cids, ncont, c,
                               err);
        else
            hipLaunchKernelGGL(rd_lookup_kernel<7>, g, dim3(256), 0, st, dig, n, tab, log2cap, tag_mask, cids, ncont, c,
                               err);
        hipLaunchKernelGGL(rd_scan_kernel, dim3(1), dim3(1024), 0, st, c, n, total);
    } else {
        hipLaunchKernelGGL(rd_gather_kernel, dim3((n + 3) / 4), dim3(256), 0, st, c, n, bases, out);
    }
    return hipGetLastError();
}

size_t rd_chunk_bytes() { return sizeof(RdChunk); }

hipError_t launch_gx_locate(int hasher, const uint32_t *dig, int n, const IndexEntry *tab, int log2cap,
                            unsigned long long tag_mask, int G, int rank, uint32_t *loc, int *err, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    const dim3 g((n + 255) / 256);
    if (hasher == 0)
        hipLaunchKernelGGL(gx_locate_kernel<5>, g, dim3(256), 0, st, dig, n, tab, log2cap, tag_mask, G, rank, loc, err);
    else
        hipLaunchKernelGGL(gx_locate_kernel<7>, g, dim3(256), 0, st, dig, n, tab, log2cap, tag_mask, G, rank, loc, err);
    return hipGetLastError();
}

// gather a host-built chunk list (RdChunk {base index, start, len, off}) into out
hipError_t launch_rd_gather(const void *chunks, int n, const uint64_t *bases, uint8_t *out, hipStream_t st)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(rd_gather_kernel, dim3((n + 3) / 4), dim3(256), 0, st, (const RdChunk *)chunks, n, bases, out);
    return hipGetLastError();
}

}  // namespace hdrf
