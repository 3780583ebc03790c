// launchers.hpp — host-side kernel launchers shared by api.hip (one stream per context).
#pragma once
#include "common.hpp"

namespace hdrf {

// Stage markers: when timing is on, a HIP event is recorded on the launch stream at every
// stage boundary (kernels of one stream run in order, so event deltas are kernel times).
// walk, stitch, sha, (unused), claim, apply, slow+decide, scan, flush, place, compress, gmax, then the
// node-global phases: local aggregation, owner, decide, flush function, allocator scan, placement,
// commit, and the X1 / X2 / descriptor all-gather / X3 exchanges (api.hip gx_collect)
constexpr int kNumStages = 23;
struct Marker {
    hipEvent_t *ev = nullptr;   // kNumStages + 1 events
    int next = 0;
    __host__ void mark(hipStream_t st)
    {
        if (ev) (void)hipEventRecord(ev[next], st);
        next++;
    }
};

struct StoreParams {
    int nblocks, cap_blk, ntiles;
    int n_thread, min_mt;      // DataDeduplicator.nThread (3), small-block threshold (25)
    uint32_t cmax;             // DataDeduplicator.maxSize
    uint32_t nslots;           // container arena slots
    int ev_cap;                // flush events per range per batch
    int closed_cap;            // closed containers per batch
    int place_lds = 0;         // dynamic LDS per place workgroup (occupancy throttle, 0 = none)
    int place_deep = 0;        // place copies 4 (1) or 2 (0) 16-B words per thread in flight (HDRF_PLACE_DEEP)
};

// chunking: granule maxima -> lane walk (total_waves waves over the batch's segments) -> repair ->
// stitch -> fallback.  gm: [nblocks][gstride] bytes, gstride >= max_len / 16 + 4 * 128.
int lane_spec_cap(int seg_len, int w);
// scratch of one batch's chunking (api.hip slot buffers)
struct ChunkScratch {
    uint8_t *gm;             // granule maxima [nblocks][gstride]
    int gstride;
    int *rq, *rq_count;      // repair queue (rq_cap entries)
    int rq_cap;
    uint32_t *rqkeep;        // [kRqKeep][64]: the cuts a repair walk found, when it found at most 63 before
                             // the shared one (the emit pass copies them instead of walking again)
    uint32_t *irr;           // irregular-boundary bitmask over the batch's segments (+2 words)
    PathInfo *path;          // [nblocks]
    int *jx;                 // [nblocks][jcap] on-path jump sources
    uint32_t *jt;            // [nblocks][jcap] targets | shared-cut index << 24
    int jcap;                // jumps per block (>= its segment boundaries)
    uint32_t *wgsum;         // [nblocks][maxw] piece sums per 256 segments
    int maxw;
    int ring = 1;            // lane walk: granule maxima through the LDS ring (off beside LZ4 passes)
};
int setprio_mask();   // HDRF_SETPRIO (chunk.hip)
// The fused chunk + fingerprint pass (lanehash.hip, HDRF_FUSED=1): its digest outputs.
struct FusedFront {
    int hasher;
    uint32_t *sdig;          // [segments][spec_cap][HW]: the digest of every cut of a lane's chain
    uint32_t *bdig;          // [segments][HW]: the chunk ending at the cut where lane k met segment k + 1
    uint32_t *dig;           // the batch's digest rows [nblocks][cap_blk][HW]
    uint8_t *need;           // [nblocks][cap_blk]: 1 = left to the fix-up hash (launch_sha_need)
    int *gm_need;            // [nblocks]: a boundary of the block went to the repair walk (granule maxima)
};
hipError_t launch_chunking(const BlockDesc *d_blocks, int nblocks, int64_t max_len, int max_nseg, int total_waves,
                           int nsegs, const ChunkScratch &X, int w, int maxlen, uint32_t *spec, int spec_cap,
                           SegMeta *meta, BlockState *bst, uint32_t *offsets, int cap_blk, int *err, hipStream_t st,
                           Marker *mk, hipStream_t stg = nullptr, hipEvent_t gdone = nullptr,   // stg: gmax pass stream
                           const FusedFront *fz = nullptr);
hipError_t launch_lane_hash(int hasher, const BlockDesc *d_blocks, int nblocks, int total_waves, int w, int maxlen,
                            uint32_t *spec, int cap, SegMeta *meta, int *rq, int *rq_count, int rq_cap, uint32_t *irr,
                            uint32_t *sdig, uint32_t *bdig, int *gm_need, int *err, hipStream_t st);
// the fused pass's fix-up: the chunks whose need[] byte is set, compacted into list (nblocks x cap_blk)
hipError_t launch_sha_need(int hasher, const BlockDesc *d_blocks, int nblocks, const uint32_t *offsets,
                           const BlockState *bst, int cap_blk, uint32_t *digests, uint32_t *queue, const uint8_t *need,
                           uint32_t *list, hipStream_t st, Marker *mk);
hipError_t launch_sha(int hasher, const BlockDesc *d_blocks, int nblocks, const uint32_t *offsets,
                      const BlockState *bst, int cap_blk, uint32_t *digests, uint32_t *queue, bool long_lanes,
                      hipStream_t st, Marker *mk);   // queue: 65 words; [64] = long chunks seen
hipError_t launch_index_load(int hasher, const uint32_t *dw, const uint8_t *vals, int n, IndexEntry *tab, int log2cap,
                             unsigned long long key, uint32_t bload, int *err, hipStream_t st);
// GzipCodec read side (inflate.hip): one raw deflate stream -> dst; res[0] = length or < 0, res[1] =
// bytes consumed.  CRC-32 of fixed-size pieces of a buffer.
int64_t inflate_chunks(int64_t slen);
hipError_t launch_inflate_find(const uint8_t *src, int64_t slen, int64_t *starts, int64_t *info, hipStream_t st);
hipError_t launch_inflate_write(const uint8_t *src, int64_t slen, const int64_t *jobs, int njobs, uint32_t *scratch,
                                int64_t cap, int *err, hipStream_t st);
hipError_t launch_inflate_resolve(uint32_t *scratch, int64_t n, unsigned int *left, hipStream_t st);
hipError_t launch_inflate_pack(const uint32_t *scratch, int64_t n, uint8_t *dst, hipStream_t st);
struct CrcOp { uint32_t m[32]; };       // GF(2) operator "append k zero bytes" (columns)
hipError_t launch_crc32_pieces(const uint8_t *data, int64_t n, const CrcOp &op1k, uint32_t *crc, hipStream_t st);
hipError_t launch_index_probe(int hasher, const BlockState *bst, int nblocks, int cap_blk, const uint32_t *digests,
                              const uint32_t *slot, int log2cap, unsigned long long key,
                              unsigned long long *stats, hipStream_t st);
// (log2cap < 0: only the allocator seed; a reset that bumps the index epoch)
hipError_t launch_index_clear(IndexEntry *tab, int log2cap, AllocState *d_alloc, const AllocState &a, hipStream_t st,
                              uint32_t ring_per = 0);
hipError_t launch_index(int hasher, const BlockState *bst, int nblocks, int cap_blk, const uint32_t *offsets,
                        const uint32_t *digests, IndexEntry *tab, int log2cap, uint32_t cur, uint32_t bfirst,
                        unsigned long long key, uint32_t *slot,
                        uint32_t *coll, uint32_t *ncoll, int coll_cap, uint8_t *flags, uint32_t *tilesum,
                        int ntiles, int *err, hipStream_t st, Marker *mk, uint8_t *dcnt = nullptr);
// (dcnt: idx_finalize follows and hands place the designated chunks; decide settles the chunks
//  without repeats in their min block itself)
// node-global index mode (gx.hip): place_kernel emits (owner slot, cid, start, stop) for new entries
struct GxPlace {
    const uint32_t *x2 = nullptr;          // owner responses, indexed by scratch IndexEntry::cid
    uint32_t *x3 = nullptr;                // [G][cap][4] location records (nullptr: classic mode)
    int64_t cap = 0;
    unsigned long long *counts = nullptr;  // [G]
    int G = 1;
    int part = 0;                          // 0 the whole place pass; 1 placement + index/X3 writes only
                                           // (no arena copy); 2 the arena copy only (node-global split)
};
// Node-global allocator scan on the device (store.hip): this rank's flush function packed into a
// fixed-size descriptor (gx_fn_bytes), and the composition of every rank's descriptor (rank order)
// from the node's allocator after the previous batch.
struct GxFnHead {            // descriptor header (the rows follow, per range t < 3: mcap x GxFnRow)
    uint64_t n_thread, mcap;
    uint64_t any[4], S[4], base_last[4], S_last[4], m[4];
};
struct GxFnRow {             // first close point v (stream prefix), fill after the batch S - cs, closes - 1
    uint32_t v, cur, n, pad;
};
uint64_t gx_fn_mcap(uint32_t cmax, int window, int max_batch);
uint64_t gx_fn_bytes(uint32_t cmax, int window, int max_batch);
hipError_t launch_fn_pack(int n_thread, const FnRange *fr, const uint64_t *rows, int64_t kcap,
                          const unsigned long long *K, uint64_t mcap, void *desc, int *err, hipStream_t st);
// states[0] = this rank's allocator in, [1] its predicted flush result, [2] the node's after the batch;
// `alloc` (the node's state after the previous batch) becomes states[0]
hipError_t launch_gx_scan(const void *descs, uint64_t fn_bytes, int G, int rank, int n_thread, uint32_t per,
                          uint32_t cmax, AllocState *alloc, AllocState *states, int *err, hipStream_t st);

hipError_t launch_store(const StoreParams &P, const BlockDesc *d_blocks, const BlockState *bst,
                        const uint32_t *offsets, const uint8_t *flags, const uint32_t *tilesum, uint32_t *tilepre,
                        uint64_t *store_size, uint32_t *pre, AllocState *alloc, RangeState *rstate, FlushEv *events,
                        ClosedRec *closed, uint32_t *nclosed, const uint32_t *slot, IndexEntry *tab, uint8_t *arena,
                        uint32_t *place_cid, uint32_t *place_pos, int *err, hipStream_t st, Marker *mk,
                        const GxPlace *gx = nullptr, const uint8_t *dcnt = nullptr);
// flush only / place only (the node-global mode chains the flush walk across ranks)
hipError_t launch_store_scan(const StoreParams &P, const BlockState *bst, const uint32_t *offsets, const uint8_t *flags,
                             const uint32_t *tilesum, uint32_t *tilepre, uint64_t *store_size, uint32_t *pre,
                             hipStream_t st);
hipError_t launch_flush_fn(const StoreParams &P, const BlockState *bst, const uint64_t *store_size, const uint32_t *pre,
                           FnBlock *fb, FnRange *fr, uint64_t *out, int64_t kcap, unsigned long long *K, int *err,
                           hipStream_t st);
hipError_t launch_store_flush(const StoreParams &P, const BlockState *bst, const uint64_t *store_size, const uint32_t *pre,
                              AllocState *alloc, RangeState *rstate, FlushEv *events, ClosedRec *closed,
                              uint32_t *nclosed, int *err, hipStream_t st);
hipError_t launch_store_place(const StoreParams &P, const BlockDesc *d_blocks, const BlockState *bst,
                              const uint32_t *offsets, const uint8_t *flags, const uint32_t *pre,
                              const RangeState *rstate, const FlushEv *events, const uint32_t *slot, IndexEntry *tab,
                              uint8_t *arena, uint32_t *place_cid, uint32_t *place_pos, const GxPlace &gx,
                              hipStream_t st, const uint8_t *dcnt = nullptr);
// designated chunk, its block count and the cleared batch-local entry state, after decide (index.hip)
hipError_t launch_index_finalize(const BlockState *bst, int nblocks, int cap_blk, int ntiles, IndexEntry *tab,
                                 const uint32_t *slot, uint8_t *flags, uint8_t *dcnt, hipStream_t st);
hipError_t launch_gx_emit(int hasher, const BlockState *bst, int nblocks, int cap_blk, int ntiles,
                          const uint32_t *digests, IndexEntry *scratch, const uint32_t *slot, const uint8_t *flags,
                          uint32_t gbase, int G, uint32_t *x1, int64_t cap, unsigned long long *counts, int *err,
                          hipStream_t st);
hipError_t launch_gx_owner(int hasher, const uint32_t *x1, const int64_t *counts, int64_t max_count, int64_t cap, int G,
                           IndexEntry *tab, int log2cap, uint32_t cur, uint32_t bfirst, unsigned long long key, uint32_t *oslot,
                           uint8_t *oflags, uint32_t *coll, uint32_t *ncoll, int coll_cap, uint32_t *x2,
                           unsigned long long *x3exp, int *err, hipStream_t st);
hipError_t launch_gx_decide(const BlockState *bst, int nblocks, int cap_blk, int ntiles, const uint32_t *offsets,
                            const IndexEntry *scratch, const uint32_t *slot, const uint32_t *x2, uint8_t *flags,
                            uint32_t *tilesum, hipStream_t st);
hipError_t launch_gx_x3want(const uint32_t *x2, const unsigned long long *sent, int64_t max_sent, int64_t cap, int G,
                            unsigned long long *want, hipStream_t st);
hipError_t launch_gx_commit(const uint32_t *x3, const int64_t *counts, int64_t max_count, int64_t cap, int G,
                            IndexEntry *tab, int log2cap, int *err, hipStream_t st);
// recipes (storeDB): a batch's digests copied into the device recipe store
struct RecipeCopy {
    uint64_t src, dst;       // device addresses (4-B aligned)
    uint32_t words, pad;
};
hipError_t launch_recipe_copy(const RecipeCopy *jobs, int n, hipStream_t st);
// device -> device-mapped (pinned) host copies on the CUs (container drain)
struct XferJob {
    uint64_t src, dst, n;
};
hipError_t launch_xfer(const XferJob *jobs, int n, uint64_t max_bytes, int wgs, hipStream_t st);
// stream mode (compressor 4): pieces of one block -> LZ4 blocks (stage) -> framed file
struct LzPiece {
    uint64_t src;            // offset in the block
    uint32_t len;            // <= 261,100
    uint32_t pad;
};
struct LzOut {
    uint64_t dst;            // offset of the piece's bytes in the file
    uint32_t hval;           // BE32 word before the size word (raw length), if hlen == 4
    uint32_t hlen;           // 0 or 4
};
hipError_t launch_lz4_stream(const LzPiece *pieces, int n, const uint8_t *base, uint8_t *stage, uint32_t *clen,
                             hipStream_t st);
hipError_t launch_lz4_emit(const LzOut *outs, int n, const uint8_t *stage, const uint32_t *clen, uint8_t *file,
                           hipStream_t st);
uint64_t lz4_piece_stride();
struct LzDec {               // one LZ4 block of a Lz4Codec file -> raw bytes
    uint64_t src, dst;       // offsets in the file / in the output
    uint32_t clen, rawlen;
};
hipError_t launch_lz4_decode(const LzDec *items, int n, const uint8_t *src, uint8_t *dst, int *err, hipStream_t st);
// stream mode compressor 3 (lzo.hip): LzopCodec blocks (LZO1X-1, raw when not smaller) at stage +
// i * lzo_piece_stride(); the decoder for LzopCodec files
hipError_t launch_lzo_stream(const LzPiece *pieces, int n, const uint8_t *base, uint8_t *stage, uint32_t *clen,
                             hipStream_t st);
hipError_t launch_lzo_decode(const LzDec *items, int n, const uint8_t *src, uint8_t *dst, int *err, hipStream_t st);
uint64_t lzo_piece_stride();
// stream mode compressor 0 (snappy.hip): pieces (pad = first fragment) split into 64 KiB
// fragments -> raw snappy groups at stage + i * stride; decoder for SnappyCodec files
hipError_t launch_snappy_stream(const LzPiece *pieces, int n, const LzPiece *frags, int nf, const uint8_t *base,
                                uint8_t *scratch, uint32_t *fclen, uint8_t *stage, uint64_t stride, uint32_t *clen,
                                hipStream_t st);
uint64_t snappy_frag_stride();
// stream mode compressor 5 (gzip.hip), stage 1 of the GPU deflate: per-position chain-128 /
// chain-32 longest_match answers ((len << 16) | dist); prev = n u32 scratch
hipError_t launch_gzip_match(const uint8_t *src, int64_t n, uint32_t *prev, uint32_t *out128, uint32_t *out32,
                             hipStream_t st);
size_t gzip_parse_scratch(int64_t n);
hipError_t launch_gzip_parse(const uint8_t *src, int64_t n, const uint32_t *m128, const uint32_t *m32, uint32_t *syms,
                             int64_t *blks, int64_t *cnt, void *scratch, hipStream_t st);
size_t gzip_block_state_bytes();
size_t gzip_tab_bytes();
void gzip_host_tab(void *dst);
hipError_t launch_gzip_encode(const uint8_t *src, int64_t n, const void *tab, const uint32_t *syms, const int64_t *blks,
                              int nblk, void *state, uint8_t *scratch, int64_t slot, int64_t *info, int64_t *off,
                              uint32_t *pcrc, uint8_t *out, int64_t *flen, hipStream_t st);
hipError_t launch_snappy_decode(const LzDec *items, int n, const uint8_t *src, uint8_t *dst, int *err, hipStream_t st);
// compression stage (lz4.hip): closed containers -> Lz4Codec files in the compressed arena
uint64_t lz4_slot_bytes(uint32_t cmax);
hipError_t launch_lz4(const ClosedRec *closed, const uint32_t *nclosed, int closed_cap, uint32_t cmax,
                      const uint8_t *arena, uint8_t *carena, uint64_t cslot, uint32_t *seg_clen, uint32_t *file_len,
                      uint32_t *work, hipStream_t st);
// read side (read.hip): lookup + scan (gather = false), then the copy (gather = true)
size_t rd_chunk_bytes();
hipError_t launch_gx_locate(int hasher, const uint32_t *dig, int n, const IndexEntry *tab, int log2cap,
                            unsigned long long key, int G, int rank, uint32_t *loc, int *err, hipStream_t st);
hipError_t launch_rd_gather(const void *chunks, int n, const uint64_t *bases, uint8_t *out, hipStream_t st);
hipError_t launch_reconstruct(int hasher, const uint32_t *dig, int n, const IndexEntry *tab, int log2cap,
                              unsigned long long key, const uint32_t *cids, const uint64_t *bases, int ncont,
                              void *chunks, uint64_t *total, uint8_t *out, int *err, hipStream_t st, bool gather);
hipError_t launch_corpus(uint8_t *dev, const uint32_t *d_roots, int64_t nblocks, int64_t spb, int64_t seg_bytes,
                         uint64_t seed, int mixed, hipStream_t st);

}  // namespace hdrf
