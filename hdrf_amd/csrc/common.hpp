// common.hpp — shared device helpers and on-device layouts for libhdrf (gfx950 only).
//
// Data layout in HBM (one batch of up to 64 blocks):
//   block bytes          caller's device buffers (16-B aligned), `readable` bytes each
//   spec lists           [block][segment][SPEC_CAP] u32 cut offsets from the speculative walk
//   offsets              [block][cap_blk] u32 chunk END offsets (reference chunking() output)
//   digests              [block][cap_blk][H] bytes
//   chunk meta           [block][cap_blk] slot / flags / prefix
//   index table          2^k entries x 64 B, open addressing keyed by the first 8 digest bytes
//   container arena      slots x container_max bytes (raw containers, DataDeduplicator.maxSize)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hdrf {

#define HDRF_GLOBAL_FWD __attribute__((address_space(1)))
constexpr int kWave = 64;
constexpr int kMaxBatch = 64;        // one bit per block of the batch in IndexEntry::mask
// Lane walker (chunk.hip): one lane walks one speculative segment of seg_len bytes; a wave holds
// kWaveSegs segments plus a helper lane that walks the next wave's first segment.
constexpr int kWaveSegs = 63;
constexpr int kLaneOver = 8;         // overrun cuts a lane may record past its segment end
constexpr int kLdsCuts = 30;         // LDS list of every lane (u16 offsets from its segment start)
constexpr int kRepairCuts = 4096;    // a repair walk gives up after this many cuts ...
constexpr int kRepairBytes = 2 << 20;  // ... or this many bytes past its start
constexpr int kRqKeep = 16384;       // repair-queue entries whose cuts the count pass keeps (64 words each)
constexpr int kSegMinWin = 4;        // seg_len bounds, in units of window + 2 (702 B)
constexpr int kSegMaxWin = 20;        // seg_len / 702 + 2 + kLaneOver <= kLdsCuts
// the fused chunk + fingerprint pass (lanehash.hip) sizes its segments for one round of its waves,
// which needs longer segments on a 4 GiB batch (24 windows): its own list bound
constexpr int kSegMaxWinF = 28;
constexpr int kLdsCutsF = 40;        // kSegMaxWinF + 2 + kLaneOver <= kLdsCutsF

// Index entry: 64 B.  tag = the table generation ("epoch", 1..255) in bits 56..63 over the first 7
// digest bytes; an entry whose tag carries another epoch is EMPTY, so a fresh index (hdrf_reset)
// is one epoch bump instead of 2^k x 64 B of zero stores (a real clear only every 255 resets and
// at open).  `dig` holds digest bytes 8..27; the 8th digest byte lives in dig[4] (SHA-1: dig[3..4]
// hold bytes 0..7) or in ncopy bits 8..15 (SHA-224).  ncopy (bits 0..7) / cid / start / stop are
// the 11-byte Redis value (chunkMeta.getMeta, DN/chunkMeta.java:62-77) in unpacked form.
struct alignas(64) IndexEntry {
    unsigned long long tag;
    unsigned long long mask;    // batch-local: bit b = block b of the batch holds the digest
    unsigned long long first;   // batch-local: max over ((63-b)<<32 | chunk index)
    uint32_t batch;             // batch id that created the entry (ids only grow over a context's life)
    uint32_t ncopy;             // bits 0..7 nCopy, bits 8..15 digest byte 7 (SHA-224)
    uint32_t cid;
    uint32_t start;
    uint32_t stop;
    uint32_t dig[5];

};
static_assert(sizeof(IndexEntry) == 64, "IndexEntry must be one 64-B line");

// Tag key of a table: (epoch << 56) | the tag-bit mask (all ones except under the collision test
// hook, debug_tag_bits).  tag_word: the entry tag a digest must carry; tag_live: an entry of the
// current epoch; tag_home: the digest's home slot (independent of the epoch).
constexpr unsigned long long kTag56 = 0x00FFFFFFFFFFFFFFull;
__host__ __device__ __forceinline__ unsigned long long tag_word(const uint32_t *dw, unsigned long long key)
{
    return ((((unsigned long long)dw[0] | ((unsigned long long)dw[1] << 32)) & key) & kTag56) | (key & ~kTag56);
}
__host__ __device__ __forceinline__ bool tag_live(unsigned long long t, unsigned long long key)
{
    return ((t ^ key) >> 56) == 0;
}
__host__ __device__ __forceinline__ uint64_t tag_home(unsigned long long t, int log2cap)
{
    return ((t & kTag56) * 0x9E3779B97F4A7C15ull) >> (64 - log2cap);
}
// the full digest equals the entry's (the caller matched the tag word: bytes 0..6)
template <int HW>
__host__ __device__ __forceinline__ bool entry_matches(const IndexEntry &e, const uint32_t *dw)
{
#pragma unroll
    for (int i = 2; i < HW; i++)
        if (e.dig[i - 2] != dw[i]) return false;
    if (HW == 5) return e.dig[3] == dw[0] && e.dig[4] == dw[1];
    return ((e.ncopy >> 8) & 0xffu) == (dw[1] >> 24);
}
// a claimed entry's digest bytes (nCopy is written by the chunk that SETs the value)
template <int HW>
__device__ __forceinline__ void store_dig(IndexEntry *e, const uint32_t *dw)
{
#pragma unroll
    for (int i = 2; i < HW; i++) e->dig[i - 2] = dw[i];
    if (HW == 5) { e->dig[3] = dw[0]; e->dig[4] = dw[1]; }
    else e->ncopy = (dw[1] >> 24) << 8;
}
// nCopy (bits 0..7 of ncopy) without touching the SHA-224 digest byte above it
__device__ __forceinline__ void set_ncopy(IndexEntry *e, uint32_t n)
{
    *(HDRF_GLOBAL_FWD uint8_t *)&e->ncopy = (uint8_t)n;
}

// Per-batch block descriptor (device side).
struct BlockDesc {
    const uint8_t *data;
    uint64_t len;
    uint64_t readable;       // bytes readable from data (>= len)
    int32_t nseg;            // speculative lane segments [k*seg_len, min((k+1)*seg_len, len))
    int32_t seg_len;         // multiple of 702 (window + 2) so all-zero data syncs at once
    int32_t seg0;            // the block's first segment in the batch's flat spec / meta arrays
    int32_t wave0;           // the block's first lane-walker wave
};

// Speculative segment walk result (one per lane segment).
constexpr int kSyncEnd = -1;         // the chain ran to the block end without meeting the next one
constexpr int kSyncFail = -2;        // no shared cut within the overrun caps (no repair record)
constexpr int kSyncJump = -3;        // repaired: the chain continued and met segment k + jmp at its cut jj
constexpr int kSyncGiveUp = -4;      // repair found no shared cut within kRepairCuts / kRepairBytes
struct SegMeta {
    int32_t n_main;          // cuts < next segment start
    int32_t n_over;          // cuts >= next segment start (<= kLaneOver)
    int32_t sync;            // i | j << 16: overrun cut i == the next segment's cut j; or a kSync* status
    int32_t jmp;             // kSyncJump: target segment - this segment
    int32_t jj;              // kSyncJump: index of the shared cut in the target's list
    int32_t n_ext;           // kSyncJump: cuts of the repair walk, the shared cut included
    int32_t ext_dst;         // the repair's cuts go to offsets[ext_dst..] (-1: not on the block's path)
    int32_t cp_from;         // stitch plan: copy list[cp_from, cp_from + cp_n) to the block's offsets
    int32_t cp_n;
    int32_t cp_dst;          // unused
    int32_t pad[3];          // stitch scratch: piece size, repair-cut position in the piece
};

// Stitch path of one block (stitch_path_kernel): on-path jumps, the terminal segment, fallback flag.
struct PathInfo {
    int32_t nj, term, fb, pad;
};

// Per-block state after chunking/stitching.
struct BlockState {
    int32_t n_cuts;          // true boundaries before the drop-last rule (stitched + fallback)
    int32_t fail_dst;        // fallback writes from here (-1 = none); it starts at offsets[fail_dst - 1]
                             // (or at the block start, first-chunk rule, when fail_dst == 0)
    uint32_t fail_p0;        // unused (kept for the layout)
    int32_t n_chunks;        // final chunk count (offsets list length)
};

// Container stream state per storer range t (lastBlockID[t], file length, lastBlockID[t+4]).
struct AllocState {
    uint32_t id[4];
    uint32_t cur[4];         // open container length (file length)
    uint32_t pos[4];         // lastBlockID[t+4] (bufferBB.position() of the last storing block)
    uint32_t slot[4];        // arena slot of the open container
    uint32_t next_slot;
    uint32_t nclosed;        // containers closed so far (total)
    uint32_t exists[4];      // open container file exists
    uint32_t pad;
};

// Flush event inside one (block, range): container closes before chunk `chunk`.
struct FlushEv {
    int32_t chunk;
    uint32_t new_id;
    uint32_t new_slot;
    uint32_t base;           // range-relative prefix (X0 of `chunk`)
};

struct RangeState {          // per (block, range t)
    uint32_t id0, slot0, cur0;   // open container at the range start
    int32_t nflush;              // flush events of this (block, range)
    int32_t ev_begin;            // first event in the range-t event list
    int32_t c_begin, c_end;      // chunk range [n*t/nT, n*(t+1)/nT)
    uint32_t base;               // block prefix of new bytes before c_begin
    uint32_t total;              // new bytes in range
    int32_t active;              // storer t runs (storeSize != 0 and t < nThread)
};

// Node-global allocator scan (gx.hip / api.hip hdrf_gx_flush_fn): one range's flush walk over
// a batch as a function of the open container's fill, with the batch's active blocks of range t
// laid end to end as one stream of new bytes.
struct FnBlock {             // per (range t, block b)
    uint32_t act, c0, c1, base;   // active (storeSize != 0 and t < nT), chunk range, pre[c0 - 1]
    uint64_t off, S;              // stream offset of the block's first new byte, new bytes
    uint32_t coff, pad;           // stream index of the block's first chunk
};
struct FnRange {             // per range t
    uint64_t any, S, base_last, S_last, nstream;
};

struct ClosedRec {           // a container closed during a batch
    uint32_t id, slot, len, range;
};

// ------------------------------------------------------------------------------------------
// Global-address-space views: pointers that arrive inside structs are generic (flat) to the
// compiler; flat loads also count in lgkmcnt and force vmcnt(0)-style waits.  Casting to
// address_space(1) yields global_load_* with precise vmcnt accounting.
#define HDRF_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ const HDRF_GLOBAL T *gptr(const void *p)
{
    return (const HDRF_GLOBAL T *)(p);
}
template <class T>
__device__ __forceinline__ HDRF_GLOBAL T *gptr_w(void *p)
{
    return (HDRF_GLOBAL T *)(p);
}

typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
// 16-B global load (dword-aligned address is enough on gfx950)
__device__ __forceinline__ uint4 ld16(const void *p)
{
    const u32x4v v = *(const HDRF_GLOBAL u32x4v *)(p);
    return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t ld4(const void *p) { return *(const HDRF_GLOBAL uint32_t *)(p); }
// streaming (nontemporal) 16-B load / store: bytes read or written once, kept from displacing
// the lines other stages re-read in L2 (granule maxima, SHA pairs, index entries, LZ4 windows)
__device__ __forceinline__ uint4 ld16_nt(const void *p)
{
    const u32x4v v = __builtin_nontemporal_load((const HDRF_GLOBAL u32x4v *)(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}
template <bool NT>
__device__ __forceinline__ uint4 ld16_t(const void *p) { return NT ? ld16_nt(p) : ld16(p); }

__device__ __forceinline__ int lane_id() { return __lane_id(); }
// wave index inside the workgroup, as a provably wave-uniform (scalar) value
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint32_t rdfirst(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Wave-wide unsigned max (all lanes participate; result uniform).
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
    // row_ror:1,2,4,8 -> every lane holds its 16-lane row max
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x121, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x122, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xf, 0xf, false));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xf, 0xf, false));
    uint32_t a = max(rdlane(v, 0), rdlane(v, 16));
    uint32_t b = max(rdlane(v, 32), rdlane(v, 48));
    return max(a, b);
}

// Inclusive wave prefix sum (u32) via shuffles.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v)
{
    const int l = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t t = __shfl_up(v, d, 64);
        if (l >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ unsigned long long ballot64(bool p) { return __ballot(p); }

// Reserve one slot of counter counts[d] for every lane that wants one (256 threads; every thread of
// the workgroup calls it, in uniform control flow): the lanes count in LDS, then one global atomic
// per (workgroup, counter) takes the workgroup's slots (d < G <= 64; s_cnt / s_base: LDS [64]).  The
// node-global record regions are filled through G counters, one per owner rank: one returning
// atomic per chunk on those few addresses serialised at the memory side (gx_emit 30.8 ms and place
// part 1 ~20 ms per 4 GiB batch, profiles/r06_lb2_kernel_stats.csv), one per wave still ~1.5 ms.
__device__ __forceinline__ unsigned long long wg_reserve(unsigned long long *counts, int d, bool want, int G,
                                                         uint32_t *s_cnt, unsigned long long *s_base)
{
    const int t = (int)threadIdx.x;
    if (t < G) s_cnt[t] = 0u;
    __syncthreads();
    uint32_t li = 0;
    if (want) li = atomicAdd(&s_cnt[d], 1u);
    __syncthreads();
    if (t < G && s_cnt[t]) s_base[t] = atomicAdd(counts + t, (unsigned long long)s_cnt[t]);
    __syncthreads();
    return want ? s_base[d] + li : 0ull;
}


// Bounds-checked 16-B load (bytes >= avail read as 0).
__device__ __noinline__ uint4 load16_guard(const uint8_t *base, int64_t off, int64_t avail)
{
    if (off + 16 <= avail) return ld16(base + off);
    uint32_t w[4] = {0, 0, 0, 0};
    for (int i = 0; i < 16; i++)
        if (off + i < avail) w[i >> 2] |= (uint32_t)base[off + i] << (8 * (i & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __noinline__ uint32_t load4_guard(const uint8_t *base, int64_t off, int64_t avail)
{
    if (off + 4 <= avail) return ld4(base + off);
    uint32_t w = 0;
    for (int i = 0; i < 4; i++)
        if (off + i < avail) w |= (uint32_t)base[off + i] << (8 * i);
    return w;
}

// 16 output bytes from an arbitrarily aligned source: two aligned 16-B loads + a funnel shift by
// sh = src & 15 (uniform per run, since destination words are 16-B aligned within a run).
template <bool NT = false>
__device__ __forceinline__ uint4 load16_shift(const uint8_t *src_aligned, int sh)
{
    const uint4 x = ld16_t<NT>(src_aligned);
    if (sh == 0) return x;
    const uint4 y = ld16_t<NT>(src_aligned + 16);
    const uint32_t r = (uint32_t)(sh & 3);
#define AB(hi, lo) __builtin_amdgcn_alignbyte((hi), (lo), r)
    switch (sh >> 2) {                                   // uniform per run
    case 0: return make_uint4(AB(x.y, x.x), AB(x.z, x.y), AB(x.w, x.z), AB(y.x, x.w));
    case 1: return make_uint4(AB(x.z, x.y), AB(x.w, x.z), AB(y.x, x.w), AB(y.y, y.x));
    case 2: return make_uint4(AB(x.w, x.z), AB(y.x, x.w), AB(y.y, y.x), AB(y.z, y.y));
    default: return make_uint4(AB(y.x, x.w), AB(y.y, y.x), AB(y.z, y.y), AB(y.w, y.z));
    }
#undef AB
}

__device__ __forceinline__ void st16(void *p, uint4 v)
{
    u32x4v w = {v.x, v.y, v.z, v.w};
    *(HDRF_GLOBAL u32x4v *)p = w;
}
template <bool NT>
__device__ __forceinline__ void st16_t(void *p, uint4 v)
{
    u32x4v w = {v.x, v.y, v.z, v.w};
    if (NT) __builtin_nontemporal_store(w, (HDRF_GLOBAL u32x4v *)p);
    else *(HDRF_GLOBAL u32x4v *)p = w;
}
// streaming-knob bits (HDRF_NT): 1 = granule-max pass loads, 2 = place copy loads + stores
int stream_knobs();   // default 3 (measured +1.5 % on the config-2 bench); HDRF_NT=0 turns both off

}  // namespace hdrf
