// api.hip — libhdrf C-ABI (include/hdrf.h): context, batch pipeline, host views.
//
// One context = one DataNode's reduction state on one GPU: the index table (Redis in the
// reference), the container arena (chunkDir files), the allocator ("blockID" key) and the
// recipes.
//
// Batches run as a two-stage pipeline over two HIP streams and two buffer slots:
//   front (stream A): descriptor upload, chunking, SHA            -> per-slot arrays only
//   back  (stream B): index, placement/gather, compression, read-back of the batch's small state
// Batch k's front waits only for the back of batch k-2 (its slot's previous user); its back waits
// for its own front and, by stream order, for batch k-1's back (the index, allocator and arena
// are updated strictly in block order: the reference's FIFO, DN/DataDeduplicator.java:124-158).
// So while batch k is being indexed and stored, batch k+1 is already being chunked and hashed.
// hdrf_submit_batch enqueues; hdrf_wait_batch completes the oldest batch (host bookkeeping);
// hdrf_reduce_batch does both.
#include <condition_variable>
#include <mutex>
#include <set>
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <new>
#include <string>
#include <vector>

#include "../../include/hdrf.h"
#include "launchers.hpp"

using namespace hdrf;

namespace {

constexpr int kStages = hdrf::kNumStages;
constexpr uint64_t kSlack = 64;   // readable bytes required past each block end
constexpr int kSlots = 5;         // batches in flight (walk | SHA | index+store | LZ4 passes)
constexpr int kErrCapacity = 2 | 4 | 8 | 16 | 32;  // device error bits that mean "a buffer is too small"

struct ContainerInfo {
    uint32_t slot;
    uint32_t len;
    int closed;
    uint32_t clen;           // compressor 2, closed: Lz4Codec file length (compressed arena slot)
};

// Per-batch buffers (device) and read-back (pinned host) of one pipeline slot.
struct Slot {
    BlockDesc *d_blocks = nullptr;
    uint32_t *d_spec = nullptr;
    SegMeta *d_meta = nullptr;
    // the fused front (HDRF_FUSED=1, lanehash.hip): per-cut and per-boundary digests, fix-up marks
    uint32_t *d_sdig = nullptr, *d_bdig = nullptr, *d_nlist = nullptr;
    int *d_gmneed = nullptr;
    uint8_t *d_need = nullptr;
    size_t sdig_words = 0, bdig_segs = 0;
    uint8_t *d_gm = nullptr;                  // granule maxima [B][gstride] (chunking pass 1)
    int gstride = 0;
    int64_t max_len = 0;                      // longest block of the batch in this slot
    int max_nseg = 0;                         // most segments of one block of the batch
    uint32_t *d_irr = nullptr;                // irregular-boundary bitmask (meta_cap / 32 + 2 words)
    PathInfo *d_path = nullptr;               // [B]
    int *d_jx = nullptr;                      // [B][jcap]
    uint32_t *d_jt = nullptr;                 // [B][jcap]
    int jcap = 0;
    uint32_t *d_wgsum = nullptr;              // [B][maxw_cap]
    int maxw_cap = 0;
    int *d_rq = nullptr, *d_rq_count = nullptr;   // failed speculative boundaries (repair queue), meta_cap entries
    uint32_t *d_rqkeep = nullptr;             // [kRqKeep][64] cuts of the short repair walks
    size_t spec_words = 0, meta_cap = 0;      // capacity of d_spec (u32) / d_meta (segments), grown on demand
    int total_waves = 0, total_segs = 0, spec_cap = 0;   // lane walk of the batch in this slot
    BlockState *d_bst = nullptr;
    uint32_t *d_off = nullptr, *d_dig = nullptr, *d_slot = nullptr, *d_pre = nullptr;
    uint8_t *d_flags = nullptr;
    uint8_t *d_dcnt = nullptr;                // designated chunks: blocks of the batch holding the digest
    uint32_t *d_tilesum = nullptr, *d_tilepre = nullptr;
    uint64_t *d_store = nullptr;
    RangeState *d_rstate = nullptr;
    FlushEv *d_ev = nullptr;
    ClosedRec *d_closed = nullptr;
    uint32_t *d_nclosed = nullptr;
    uint32_t *d_coll = nullptr, *d_ncoll = nullptr;
    uint32_t *d_pcid = nullptr, *d_ppos = nullptr, *d_queue = nullptr;
    uint32_t *d_segclen = nullptr, *d_filelen = nullptr;
    uint32_t *d_lzwork = nullptr;             // compressor 2: the LZ4 pass's two item counters
    int *d_err = nullptr;
    // pinned read-back, filled by stream B before back_done
    BlockState *h_bst = nullptr;
    uint64_t *h_store = nullptr;
    AllocState *h_alloc = nullptr;
    int *h_err = nullptr;
    uint32_t *h_nclosed = nullptr;
    uint32_t *h_long = nullptr;               // the batch held chunks for the long SHA lanes (queue[64])
    ClosedRec *h_closed = nullptr;
    uint32_t *h_filelen = nullptr;
    BlockDesc *h_desc = nullptr;
    // host metadata of the batch in this slot
    std::vector<uint64_t> ids, lens;
    int nblocks = 0;
    bool pending = false;
    uint32_t close_bound = 0;                 // durable containers: closes this batch may make per range
    uint32_t lz_bound = 0;                    // compressor 2: closes this batch may make per range (LZ4 lag)
    hipEvent_t placed = nullptr;              // compressor 2: the batch's place kernel finished (stream B2)
    hipEvent_t idx_done = nullptr;            // index stage (claim .. finalize) of the batch done (stream B)
    hipEvent_t lz_done = nullptr;             // compressor 2: its closed containers are Lz4Codec files
    uint32_t rx_release = 0;                  // packet path: receive buffers (bit mask) freed when the batch completes
    uint32_t gx_batch = 0;                    // node-global: index batch id of the batch in this slot
    bool gx_compressed = false;               // node-global compressor 2: hdrf_gx_compress ran for the batch
    RecipeCopy *h_rjobs = nullptr, *d_rjobs = nullptr;   // recipe copies of the batch (storeDB)
    hipEvent_t recipe_done = nullptr;         // the copies read d_dig: the slot's next SHA waits
    bool recipe_pending = false;
    bool gen_reset = false;                   // the batch starts a fresh index generation (hdrf_reset_async)
    hipEvent_t walk_done = nullptr, front_done = nullptr, back_done = nullptr, gmax_done = nullptr;
    hipEvent_t copy_done = nullptr;          // host path: the batch's H2D copies landed
    uint8_t *d_hstage = nullptr;              // host path: device copies of the batch's blocks
    uint64_t hstage_stride = 0;
    hipEvent_t evW[4] = {}, evA[3] = {}, evB[10] = {};   // stage markers (timing)
    // node-global mode: the slot's host side of a batch (pinned: front counts, count uploads, the
    // place read-back), whether a batch used the slot, and whether its arena copy ran on stream B2
    struct GxHost *h_gx = nullptr;
    std::vector<int64_t> gx_c1;               // X1 send counts of the batch in the slot
    bool gx_inuse = false, gx_split = false;
    hipEvent_t gx_meta = nullptr;             // placement (part 1) and its read-back done (stream B)
};

// Pinned per-slot exchange with the host in node-global mode: what hdrf_gx_front_wait and
// hdrf_gx_place_wait read, and the receive counts hdrf_gx_owner / hdrf_gx_commit upload (a pageable
// source would make hipMemcpyAsync wait for the stream).
struct GxHost {
    unsigned long long front_cnt[64];         // X1 records emitted per owner (gx_emit)
    int front_err, commit_err;
    int64_t up_r1[64], up_r3[64];             // X1 / X3 receive counts (uploads)
    unsigned long long c3[64], x3e[64], x3want[64];   // X3 send counts, X3 receive counts, X2-implied sends
    AllocState st[4];                         // [0] allocator in [1] predicted [2] node final [3] flush walk result
};

// Per-batch timing of the node-global phases (cfg.timing): HIP events on the streams each phase runs
// on, in a ring indexed by the batch's sequence number, collected once the batch has completed.
enum GxEv {
    kW0 = 0, kA0 = 4, kX0 = 7, kG0 = 11, kG1, kG2, kG3, kG4, kG5, kG6, kG7, kG8, kG9, kG10, kG11, kG12, kG13,
    kP0, kP1, kGxEv
};
constexpr int kGxRing = 8;
struct GxTime {
    hipEvent_t ev[kGxEv] = {};
    uint32_t rec = 0;                         // bit e: ev[e] was recorded for this batch
};

}  // namespace

struct hdrf_ctx {
    hdrf_cfg cfg{};
    int H = 20, HW = 5;
    hipStream_t st = nullptr;    // stream A: SHA stage (also every synchronous helper)
    hipStream_t stB = nullptr;   // stream B: back stage, index part (and the node-global phases)
    hipStream_t stB2 = nullptr;  // stream B2: back stage, store part (scan, flush, place, read-back)
    hipStream_t stW = nullptr;   // stream W: chunking stage
    hipStream_t stG = nullptr;   // stream G: the granule-max pass (HDRF_GMAX_STREAM), ahead of W
    hipStream_t stC = nullptr;   // stream C: H2D copies of host-submitted batches
    hipStream_t stD = nullptr;   // stream D: container drain D2H (beside the H2D copies on C)
    hipStream_t stR = nullptr;   // stream R: recipe copies once host batches use stream C (there a
                                 // kernel waited for CU slots and stalled the next batch's H2D copies)
    bool host_copies = false;    // hdrf_submit_host / hdrf_rx_begin ran: stream C carries H2D copies
    XferJob *h_xfer = nullptr;   // drain copy jobs (pinned, read by xfer_kernel)
    int xfer_cap = 0;
    hipStream_t stL[2] = {};     // compressor 2: LZ4 streams, alternating by batch (off stream B)
    // chunks >= 64 KiB were seen in the last completed batch: sha_full hashes them on dedicated
    // lanes (sha.hip); off otherwise, where the scan for them costs config 2 ~3 %
    bool sha_long = false;
    bool fused = false;                              // the fused chunk + fingerprint front (fused_front)
    int n_cu = 256;                                  // compute units of the device (the fused pass's segment sizing)
    int max_batch = 0, cap_blk = 0, ntiles = 0, ev_cap = 0, closed_cap = 0, coll_cap = 0;
    Slot sl[kSlots];
    uint64_t nsub = 0, nwait = 0;  // batches submitted / completed
    int res = 0;                   // slot of the last completed batch (hdrf_batch_* views)
    // node state (shared by all batches)
    IndexEntry *d_tab = nullptr;
    uint8_t *d_arena = nullptr;
    uint8_t *d_carena = nullptr;                 // compressor 2: Lz4Codec files of closed containers
    uint64_t cslot = 0;
    AllocState *d_alloc = nullptr;
    uint8_t *d_stage = nullptr;
    uint64_t stage_cap = 0;
    uint8_t *d_rd = nullptr;                     // reconstruction scratch (grows)
    uint64_t rd_cap = 0;
    // host state
    uint32_t batch = 0;                              // batch ids: grow over the context's life (never reset)
    uint32_t epoch = 1;                              // index generation in the tag words (1..255)
    uint32_t bfirst = 1;                             // first batch id of the current epoch
    bool gen_pending = false;                        // hdrf_reset_async: the next submit starts a generation
    bool gen_clear = false;                          //   ... whose epoch wrapped (the table is cleared)
    uint32_t scratch_epoch[kSlots] = {};             // node-global: generation of each scratch table
    int have_alloc = 0;
    int last_nblocks = 0;
    AllocState h_alloc{};
    std::map<uint32_t, ContainerInfo> containers;   // container id -> arena slot
    std::map<uint32_t, uint32_t> slot_owner;         // arena slot -> container id
    // recipes (SET longToBytes(blockId,4) -> BE32 size | digests) live in HBM: digests in an
    // append-only store of 256 MiB chunks, the host keeps only where each one is
    struct RecipeLoc { uint32_t chunk; uint64_t off; uint32_t n; };
    std::vector<uint8_t *> rchunks;
    uint32_t rcur = 0;                                // chunk being filled
    uint64_t rhead = 0;                               // bytes used in it
    std::map<uint32_t, RecipeLoc> recipes;
    std::map<uint32_t, int64_t> lengths;              // block length (recipe head)
    struct Loaded { uint8_t *ptr; uint64_t len; };
    std::map<uint32_t, Loaded> loaded;               // containers loaded back from files (read side)
    // node-global index (gx.hip): scratch aggregation table, owner-side per-record arrays
    int G = 1, rank = 0;
    // Two batches can be in the node-global pipeline: the front half of batch k+1 (slot (k+1)%2,
    // stream A) runs while batch k goes through its exchanges and back phases (slot k%2, stream B).
    IndexEntry *d_scratch[kSlots] = {};         // per-slot local aggregation table
    int scratch_log2 = 0;
    int64_t gx_cap = 0;
    int gx_depth = 3;                            // node-global batches in flight (HDRF_GX_DEPTH, 2..kSlots)
    hipStream_t stX = nullptr;                   // node-global: local aggregation + X1 records (front)
    unsigned long long *d_gxe[kSlots] = {};      // [G] X1 records emitted per peer, per slot
    unsigned long long *d_x3want = nullptr;      // [G] X3 records the X2 responses call for (sender check)
    AllocState *d_gxst = nullptr;                // [4] device allocator scan: in, predicted, node final, walk
    int *d_gx_err = nullptr;                     // errors of hdrf_gx_commit (reported by the next place / sync)
    uint64_t fn_bytes = 0, fn_mcap = 0;          // packed flush descriptor (hdrf_gx_flush_fn_dev)
    int gx_dscan = 0;                            // the back batch's allocator came from the device scan
    bool gx_place_pending = false;               // hdrf_gx_place_launch ran, hdrf_gx_place_wait not yet
    GxTime gxt[kGxRing];
    uint64_t gxt_done = 0;                       // batches whose phase times were collected
    unsigned long long *d_gx_counts = nullptr;   // [G] X3 records emitted per peer (back phases)
    int64_t *d_gx_rcounts = nullptr;             // [G] records received per peer
    // [G] X3 records each source will send this owner: one per record that holds its created entry's
    // minimum block (own_decide), so the X3 receive counts need no exchange of their own
    unsigned long long *d_gx_x3exp = nullptr;
    std::vector<int64_t> gx_x3recv;
    uint32_t *d_oslot = nullptr;
    uint8_t *d_oflags = nullptr;
    const uint32_t *gx_x2 = nullptr;             // responses of the back batch (caller's buffer)
    AllocState gx_ain{}, gx_aout{};              // allocator before / after this rank's flush walk
    AllocState gx_expect{};                      // this rank's flush result predicted by hdrf_gx_alloc_scan
    int gx_scanned = 0;                          // the back batch's allocator came from the scan
    uint8_t *d_fn = nullptr;                     // flush-function scratch (hdrf_gx_flush_fn)
    uint64_t fn_cap = 0;
    uint64_t gx_nfront = 0, gx_nfwait = 0, gx_nback = 0;   // fronts launched / waited, batches committed
    int gx_bphase = 0;                           // back batch: 0 owner next, 1 decide, 2 flush, 3 place, 4 commit
    hdrf_stats stats{};                          // cumulative since the last reset
    uint32_t lzop_mtime = 0;                     // stream codec 3: the lzop header's mtime field
    // concurrency: every entry point holds mu; ticketed reductions also wait for their turn
    // (AIWriteQueue order, DN/DataDeduplicator.java:124-158, DN/DDRunner.java:20-36)
    std::recursive_mutex mu;
    std::condition_variable_any turn;
    uint64_t next_ticket = 0, serving = 0;
    std::set<uint64_t> cancelled;
    // durable containers (cfg.retain_containers): closed containers stay in their arena slot until
    // drained; open containers' bytes already handed out
    std::vector<uint32_t> pend_closed;
    uint32_t undrained[4] = {0, 0, 0, 0};
    uint32_t inflight_bound = 0;
    uint32_t gen_reserve = 0;                 // hdrf_reset_async (durable): the old generation's open slot
    std::map<uint32_t, int64_t> handed;
    bool lost = false;
    // packet-granular receive (hdrf_rx_begin / hdrf_append_packet / hdrf_submit_slot): device
    // receive buffers, and a pinned chunk ring the packets are copied into before their H2D
    static constexpr int kRx = 16;
    // pinned staging chunk per receive buffer (two alternate): 4 MiB, HDRF_RX_CHUNK_MB for A/B
    const uint64_t kRingChunk = [] {
        const char *e = getenv("HDRF_RX_CHUNK_MB");
        const long v = e ? atol(e) : 4;
        return (uint64_t)(v >= 1 && v <= 64 ? v : 4) << 20;
    }();
    // one receive buffer per block being received: device copy of the block, and two pinned 4 MiB
    // staging chunks of its own, so receivers of different blocks (one DataXceiver thread each)
    // copy their packets concurrently, outside the context lock
    struct Rx {
        uint8_t *d = nullptr;                   // device buffer (max_block_bytes + slack)
        uint8_t *h = nullptr;                   // pinned staging, 2 x kRingChunk
        hipEvent_t ev[2] = {nullptr, nullptr};  // H2D of each staging chunk
        bool busy[2] = {false, false};
        hipStream_t st = nullptr;               // HDRF_RX_STREAMS=1: this buffer's own H2D stream
        hipEvent_t done = nullptr;              //   (its copies then never queue behind other receivers')
        int cur = 0;
        uint64_t fill = 0, dst = 0;             // bytes in the current chunk, their block offset
        uint64_t len = 0, id = 0;
        std::atomic<int> state{0};              // 0 free 1 receiving 2 submitted
    };
    Rx rx[kRx];
    bool rx_used = false;                       // a packet receive was opened (drain engine choice)
    // timing
    bool timing = false;
    double stage_ms[kStages] = {};
    std::string err;
};

#define HIPCK(x)                                                                       \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            ctx->err = std::string(#x) + ": " + hipGetErrorString(e_);                 \
            return HDRF_E_HIP;                                                         \
        }                                                                              \
    } while (0)

// every entry point: one caller at a time (a null context is checked by the function itself)
#define HDRF_LOCK(c)                                                                                 \
    std::unique_lock<std::recursive_mutex> lk_ =                                                     \
        (c) ? std::unique_lock<std::recursive_mutex>((c)->mu) : std::unique_lock<std::recursive_mutex>()

// tag key of the index (common.hpp tag_word): the current epoch over the tag-bit mask (all ones
// except under the debug_tag_bits collision hook)
static unsigned long long tag_bits(const hdrf_ctx *ctx)
{
    const int bits = ctx->cfg.debug_tag_bits;
    return ((bits <= 0 || bits >= 56) ? ~0ull : ((1ull << bits) - 1)) & kTag56;
}
static unsigned long long tag_mask(const hdrf_ctx *ctx)
{
    return ((unsigned long long)ctx->epoch << 56) | tag_bits(ctx);
}

static int set_err(hdrf_ctx *ctx, int code, const std::string &msg)
{
    if (ctx) ctx->err = msg;
    return code;
}

static int device_error(hdrf_ctx *ctx, int herr)
{
    std::string m = "device reported error flags " + std::to_string(herr);
    if (herr & 32) m += " (arena_slots too small: a storer range closed more containers in one batch than its ring holds)";
    if (herr & 2) m += " (index table full)";
    if (herr & 1) m += " (chunking: offsets capacity or an unterminated fallback walk)";
    if (herr & 192) m += " (chunking: speculative list overflow / inconsistent stitch)";
    if (herr & 4) m += " (tag-collision list full)";
    if (herr & 256) m += " (node-global: an X3 location names no index entry)";
    if (herr & 512) m += " (node-global: malformed flush descriptor in the allocator scan)";
    if (herr & 1024) m += " (node-global: flush function candidate table overflow or runaway chain)";
    return set_err(ctx, (herr & kErrCapacity) ? HDRF_E_CAPACITY : HDRF_E_DEVICE, m);
}

template <class T>
static int dalloc(hdrf_ctx *ctx, T **p, size_t count)
{
    size_t bytes = std::max<size_t>(count * sizeof(T), 256);
    if (hipMalloc((void **)p, bytes) != hipSuccess) {
        *p = nullptr;
        ctx->err = "hipMalloc failed (" + std::to_string(bytes) + " bytes)";
        return HDRF_E_NOMEM;
    }
    return 0;
}

template <class T>
static int halloc(hdrf_ctx *ctx, T **p, size_t count)
{
    if (hipHostMalloc((void **)p, std::max<size_t>(count * sizeof(T), 64), hipHostMallocDefault) != hipSuccess) {
        *p = nullptr;
        ctx->err = "hipHostMalloc failed";
        return HDRF_E_NOMEM;
    }
    std::memset(*p, 0, std::max<size_t>(count * sizeof(T), 64));
    return 0;
}

extern "C" int hdrf_default_cfg(hdrf_cfg *cfg)
{
    if (!cfg) return HDRF_E_INVAL;
    std::memset(cfg, 0, sizeof *cfg);
    cfg->hasher = 0;
    cfg->compressor = 1;
    cfg->window = 700;
    cfg->max_chunk = 1000000;
    cfg->n_thread = 3;
    cfg->min_mt_chunks = 25;
    cfg->container_max = 1u << 25;
    cfg->device = 0;
    cfg->max_block_bytes = 128ll << 20;
    cfg->max_batch_blocks = 8;
    cfg->retain_containers = 0;
    cfg->index_log2 = 22;
    cfg->arena_slots = 16;
    cfg->segment_bytes = 1 << 20;
    cfg->keep_recipes = 1;
    cfg->timing = 0;
    cfg->n_ranks = 1;
    cfg->rank = 0;
    return 0;
}

static void free_slot(Slot &S)
{
    void *dev[] = {S.d_blocks, S.d_spec, S.d_meta, S.d_gm, S.d_irr, S.d_path, S.d_jx, S.d_jt, S.d_wgsum, S.d_rq, S.d_rq_count, S.d_rqkeep, S.d_bst, S.d_off, S.d_dig, S.d_slot,
                   S.d_pre, S.d_flags, S.d_dcnt, S.d_tilesum, S.d_tilepre, S.d_store, S.d_rstate, S.d_ev, S.d_closed,
                   S.d_nclosed, S.d_coll, S.d_ncoll, S.d_pcid, S.d_ppos, S.d_queue, S.d_segclen, S.d_filelen, S.d_err,
                   S.d_lzwork, S.d_sdig, S.d_bdig, S.d_need, S.d_nlist, S.d_gmneed};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    void *host[] = {S.h_bst, S.h_store, S.h_alloc, S.h_err, S.h_nclosed, S.h_long, S.h_closed, S.h_filelen, S.h_desc,
                    S.h_gx};
    for (void *p : host)
        if (p) (void)hipHostFree(p);
    hipEvent_t evs[] = {S.walk_done, S.front_done, S.back_done, S.copy_done, S.recipe_done, S.placed, S.lz_done,
                        S.gmax_done, S.idx_done, S.gx_meta};
    if (S.d_rjobs) (void)hipFree(S.d_rjobs);
    if (S.h_rjobs) (void)hipHostFree(S.h_rjobs);
    if (S.d_hstage) (void)hipFree(S.d_hstage);
    for (auto e : evs)
        if (e) (void)hipEventDestroy(e);
    for (auto e : S.evW)
        if (e) (void)hipEventDestroy(e);
    for (auto e : S.evA)
        if (e) (void)hipEventDestroy(e);
    for (auto e : S.evB)
        if (e) (void)hipEventDestroy(e);
}

static void free_all(hdrf_ctx *ctx)
{
    for (auto &S : ctx->sl) free_slot(S);
    for (auto &kv : ctx->loaded) (void)hipFree(kv.second.ptr);
    ctx->loaded.clear();
    for (auto p : ctx->rchunks) (void)hipFree(p);
    ctx->rchunks.clear();
    void *ptrs[] = {ctx->d_tab, ctx->d_arena, ctx->d_alloc, ctx->d_stage, ctx->d_rd, ctx->d_gx_counts,
                    ctx->d_gx_rcounts, ctx->d_oslot, ctx->d_oflags, ctx->d_carena, ctx->d_fn, ctx->d_gx_x3exp,
                    ctx->d_x3want, ctx->d_gxst, ctx->d_gx_err};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    for (int i = 0; i < kSlots; i++) {
        if (ctx->d_scratch[i]) (void)hipFree(ctx->d_scratch[i]);
        if (ctx->d_gxe[i]) (void)hipFree(ctx->d_gxe[i]);
    }
    for (auto &T : ctx->gxt)
        for (auto e : T.ev)
            if (e) (void)hipEventDestroy(e);
    if (ctx->stX) (void)hipStreamDestroy(ctx->stX);
    if (ctx->st) (void)hipStreamDestroy(ctx->st);
    if (ctx->stB) (void)hipStreamDestroy(ctx->stB);
    if (ctx->stB2) (void)hipStreamDestroy(ctx->stB2);
    if (ctx->stW) (void)hipStreamDestroy(ctx->stW);
    if (ctx->stG) (void)hipStreamDestroy(ctx->stG);
    if (ctx->stC) (void)hipStreamDestroy(ctx->stC);
    if (ctx->stD) (void)hipStreamDestroy(ctx->stD);
    if (ctx->stR) (void)hipStreamDestroy(ctx->stR);
    if (ctx->h_xfer) (void)hipHostFree(ctx->h_xfer);
    for (auto L : ctx->stL)
        if (L) (void)hipStreamDestroy(L);
    for (auto &r : ctx->rx)
        if (r.d) (void)hipFree(r.d);
    for (auto &r : ctx->rx) {
        if (r.h) (void)hipHostFree(r.h);
        for (auto e : r.ev)
            if (e) (void)hipEventDestroy(e);
        if (r.done) (void)hipEventDestroy(r.done);
        if (r.st) (void)hipStreamDestroy(r.st);
    }
}

static int alloc_slot(hdrf_ctx *ctx, Slot &S)
{
    const hdrf_cfg &c = ctx->cfg;
    const int B = ctx->max_batch;
    const size_t nchunk = (size_t)B * ctx->cap_blk;
    const int nseg_lz = (int)((c.container_max + 261099) / 261100);
    int rc = 0;
    // speculative lists: sized for one wave of lane segments per 1 MiB of the largest batch, grown
    // on demand when a batch cuts finer (prepare_blocks)
    const int seg_len0 = std::max(kSegMinWin, std::min(kSegMaxWin, (int)(c.segment_bytes / kWaveSegs / (c.window + 2)))) *
                         (c.window + 2);
    S.meta_cap = (size_t)B * (size_t)(c.max_block_bytes / seg_len0 + 2);
    S.spec_words = S.meta_cap * (size_t)lane_spec_cap(seg_len0, c.window);
    S.gstride = (int)(((c.max_block_bytes + 15) / 16 + 1024 + 255) & ~(int64_t)255);
    // on-path stitch jumps: at most one per segment boundary at the finest segmentation
    S.jcap = (int)(c.max_block_bytes / ((int64_t)kSegMinWin * (c.window + 2)) + 2);
    if ((rc = dalloc(ctx, &S.d_blocks, B)) || (rc = dalloc(ctx, &S.d_spec, S.spec_words)) ||
        (rc = dalloc(ctx, &S.d_gm, (size_t)B * S.gstride)) || (rc = dalloc(ctx, &S.d_path, B)) ||
        (rc = dalloc(ctx, &S.d_jx, (size_t)B * S.jcap)) || (rc = dalloc(ctx, &S.d_jt, (size_t)B * S.jcap)) ||
        (rc = dalloc(ctx, &S.d_irr, S.meta_cap / 32 + 2)) ||
        (rc = dalloc(ctx, &S.d_meta, S.meta_cap)) || (rc = dalloc(ctx, &S.d_rq, S.meta_cap)) ||
        (rc = dalloc(ctx, &S.d_rq_count, 1)) || (rc = dalloc(ctx, &S.d_rqkeep, (size_t)kRqKeep * 64)) ||
        (rc = dalloc(ctx, &S.d_bst, B)) ||
        (rc = dalloc(ctx, &S.d_off, nchunk)) || (rc = dalloc(ctx, &S.d_dig, nchunk * ctx->HW)) ||
        (rc = dalloc(ctx, &S.d_slot, nchunk)) ||
        (rc = dalloc(ctx, &S.d_pre, nchunk)) || (rc = dalloc(ctx, &S.d_flags, nchunk)) || (rc = dalloc(ctx, &S.d_dcnt, nchunk)) ||
        (rc = dalloc(ctx, &S.d_tilesum, (size_t)B * ctx->ntiles)) ||
        (rc = dalloc(ctx, &S.d_tilepre, (size_t)B * ctx->ntiles)) || (rc = dalloc(ctx, &S.d_store, B)) ||
        (rc = dalloc(ctx, &S.d_rstate, (size_t)B * 4)) || (rc = dalloc(ctx, &S.d_ev, (size_t)3 * ctx->ev_cap)) ||
        (rc = dalloc(ctx, &S.d_closed, ctx->closed_cap)) || (rc = dalloc(ctx, &S.d_nclosed, 1)) ||
        (rc = dalloc(ctx, &S.d_coll, ctx->coll_cap)) || (rc = dalloc(ctx, &S.d_ncoll, 1)) ||
        (rc = dalloc(ctx, &S.d_pcid, nchunk)) || (rc = dalloc(ctx, &S.d_ppos, nchunk)) ||
        (rc = dalloc(ctx, &S.d_queue, 128)) || (rc = dalloc(ctx, &S.d_err, 1)) ||
        (rc = halloc(ctx, &S.h_bst, B)) || (rc = halloc(ctx, &S.h_store, B)) || (rc = halloc(ctx, &S.h_alloc, 1)) ||
        (rc = halloc(ctx, &S.h_err, 1)) || (rc = halloc(ctx, &S.h_nclosed, 1)) || (rc = halloc(ctx, &S.h_long, 1)) ||
        (rc = halloc(ctx, &S.h_closed, ctx->closed_cap)) || (rc = halloc(ctx, &S.h_filelen, ctx->closed_cap)) ||
        (rc = halloc(ctx, &S.h_desc, B)))
        return rc;
    if (c.compressor == 2 && ((rc = dalloc(ctx, &S.d_segclen, (size_t)ctx->closed_cap * nseg_lz)) ||
                              (rc = dalloc(ctx, &S.d_filelen, (size_t)ctx->closed_cap)) ||
                              (rc = dalloc(ctx, &S.d_lzwork, 2))))
        return rc;
    if ((rc = dalloc(ctx, &S.d_rjobs, B)) || (rc = halloc(ctx, &S.h_rjobs, B))) return rc;
    if (hipEventCreateWithFlags(&S.walk_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.copy_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.recipe_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.front_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.back_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.placed, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.lz_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.gmax_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.idx_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&S.gx_meta, hipEventDisableTiming) != hipSuccess)
        return set_err(ctx, HDRF_E_HIP, "hipEventCreate failed");
    for (auto &e : S.evW)
        if (hipEventCreate(&e) != hipSuccess) return set_err(ctx, HDRF_E_HIP, "hipEventCreate failed");
    for (auto &e : S.evA)
        if (hipEventCreate(&e) != hipSuccess) return set_err(ctx, HDRF_E_HIP, "hipEventCreate failed");
    for (auto &e : S.evB)
        if (hipEventCreate(&e) != hipSuccess) return set_err(ctx, HDRF_E_HIP, "hipEventCreate failed");
    if (hipMemsetAsync(S.d_err, 0, sizeof(int), ctx->st) != hipSuccess) return set_err(ctx, HDRF_E_HIP, "memset");
    return 0;
}

static int wait_one(hdrf_ctx *ctx, bool force = false);
static bool fused_front();
static int init_state(hdrf_ctx *ctx, bool fresh);
static bool gen_undrained(const hdrf_ctx *ctx);

// complete every batch in flight (views, reset, the node-global phases need a quiet context)
static int drain(hdrf_ctx *ctx)
{
    int rc = 0;
    // (forced: a generation switch whose old containers were not drained still completes, and the
    // context is marked lost until hdrf_reset)
    while (ctx->nwait < ctx->nsub)
        if (int r = wait_one(ctx, true)) rc = rc ? rc : r;
    HIPCK(hipStreamSynchronize(ctx->stC));
    if (ctx->stR) HIPCK(hipStreamSynchronize(ctx->stR));
    for (auto L : ctx->stL) HIPCK(hipStreamSynchronize(L));
    HIPCK(hipStreamSynchronize(ctx->stG));
    HIPCK(hipStreamSynchronize(ctx->stW));
    HIPCK(hipStreamSynchronize(ctx->st));
    HIPCK(hipStreamSynchronize(ctx->stB));
    HIPCK(hipStreamSynchronize(ctx->stB2));
    if (ctx->stX) HIPCK(hipStreamSynchronize(ctx->stX));
    if (rc) return rc;
    if (ctx->gen_pending && ctx->gx_nfront == ctx->gx_nback) {
        // hdrf_reset_async with no batch submitted since: the caller of a view or a restore sees the
        // fresh generation it asked for, applied now (a restore is then not undone by the next submit)
        if (ctx->cfg.retain_containers && gen_undrained(ctx))
            return set_err(ctx, HDRF_E_INVAL, "hdrf_reset_async is pending and the previous generation's containers "
                                              "were not drained (hdrf_drain_containers first, or hdrf_reset)");
        return init_state(ctx, false);
    }
    return 0;
}

static AllocState initial_alloc(const hdrf_ctx *ctx)
{
    AllocState a{};
    for (int t = 0; t < 4; t++) {
        a.id[t] = (uint32_t)t << 22;                 // utilities.bytesToBlockID, absent key (DN/utilities.java:36-50)
        // (node-global mode: the one allocator of the node, carried rank to rank by hdrf_gx_flush)
        a.slot[t] = (uint32_t)t * (uint32_t)(ctx->cfg.arena_slots / 4);   // per-range slot rings
    }
    return a;
}

// the host side of a fresh DataNode: containers, recipes, allocator view, totals
static void reset_host(hdrf_ctx *ctx)
{
    ctx->h_alloc = initial_alloc(ctx);
    ctx->have_alloc = 0;
    ctx->containers.clear();
    ctx->slot_owner.clear();
    for (auto &kv : ctx->loaded) (void)hipFree(kv.second.ptr);
    ctx->loaded.clear();
    ctx->recipes.clear();
    ctx->rcur = 0;
    ctx->rhead = 0;
    ctx->lengths.clear();
    ctx->stats = hdrf_stats{};
}

static int init_state(hdrf_ctx *ctx, bool fresh)
{
    ctx->gen_pending = false;                        // (before drain: this is the generation switch)
    (void)drain(ctx);
    const AllocState a = initial_alloc(ctx);
    for (auto &S : ctx->sl) HIPCK(hipMemsetAsync(S.d_err, 0, sizeof(int), ctx->st));
    HIPCK(hipStreamSynchronize(ctx->st));
    // the index and allocator belong to the back stream (also for the node-global back phases).
    // A fresh index is a new epoch: every entry tagged with another one is empty (common.hpp), so
    // the 2^k x 64 B table is cleared only at open and once every 255 resets; batch ids keep
    // growing, and the claim rule tells this epoch's entries by batch >= bfirst (index.hip).
    // (gen_clear: a pending hdrf_reset_async already wrapped the epoch)
    hipStream_t ist = ctx->stB;
    const bool clear = fresh || ctx->epoch >= 255 || ctx->gen_clear;
    ctx->gen_clear = false;
    ctx->epoch = clear ? 1 : ctx->epoch + 1;
    if (fresh) ctx->batch = 0;
    ctx->bfirst = ctx->batch + 1;
    HIPCK(launch_index_clear(ctx->d_tab, clear ? ctx->cfg.index_log2 : -1, ctx->d_alloc, a, ist));
    if (fresh)
        for (int i = 0; i < kSlots; i++)
            if (ctx->d_scratch[i]) {
                HIPCK(hipMemsetAsync(ctx->d_scratch[i], 0, sizeof(IndexEntry) << ctx->scratch_log2, ist));
                ctx->scratch_epoch[i] = 0;
            }
    reset_host(ctx);
    for (auto &S : ctx->sl) S.recipe_pending = S.gen_reset = false;
    ctx->last_nblocks = 0;
    ctx->gx_nfront = ctx->gx_nfwait = ctx->gx_nback = 0;
    ctx->gx_bphase = 0;
    ctx->gx_dscan = ctx->gx_scanned = 0;
    ctx->gx_place_pending = false;
    ctx->gxt_done = 0;
    for (auto &T : ctx->gxt) T.rec = 0;
    for (auto &S : ctx->sl) S.gx_inuse = S.gx_split = false;
    if (ctx->d_gx_err) HIPCK(hipMemsetAsync(ctx->d_gx_err, 0, sizeof(int), ist));
    ctx->pend_closed.clear();
    for (auto &u : ctx->undrained) u = 0;
    ctx->inflight_bound = 0;
    ctx->gen_reserve = 0;
    ctx->handed.clear();
    ctx->lost = false;
    for (auto &r : ctx->rx) { r.state = 0; r.len = 0; r.fill = 0; r.busy[0] = r.busy[1] = false; }
    for (auto &S : ctx->sl) S.rx_release = 0;
    return 0;
}

extern "C" int hdrf_open(const hdrf_cfg *cfg_in, hdrf_ctx **out)
{
    if (!cfg_in || !out) return HDRF_E_INVAL;
    *out = nullptr;
    const hdrf_cfg &c = *cfg_in;
    if ((c.hasher != 0 && c.hasher != 1) || c.window < 32 || c.window > 1000 || c.max_chunk <= c.window ||
        c.n_thread < 1 || c.n_thread > 3 || c.max_batch_blocks < 1 || c.max_batch_blocks > kMaxBatch ||
        c.index_log2 < 10 || c.index_log2 > 31 || c.arena_slots < 8 || c.max_block_bytes < 1 ||
        c.max_block_bytes > (1ll << 30) || c.container_max <= (uint32_t)c.max_chunk + 1 || c.segment_bytes < (1 << 16) ||
        c.debug_tag_bits < 0 || c.debug_tag_bits > 64 || (c.debug_tag_bits && c.hasher != 0) ||
        c.n_ranks < 1 || c.n_ranks > 64 || c.rank < 0 || c.rank >= c.n_ranks)
        return HDRF_E_INVAL;
    // 1 = dedup, 2 = dedup + Lz4Codec containers (single-node contexts; the node-global mode
    // assembles containers from several GPUs and compresses them in a later step: unsupported yet)
    if (c.compressor != 1 && c.compressor != 2) return HDRF_E_UNSUPPORTED;
    hdrf_ctx *ctx = new (std::nothrow) hdrf_ctx();
    if (!ctx) return HDRF_E_NOMEM;
    ctx->cfg = c;
    ctx->H = c.hasher == 0 ? 20 : 28;
    ctx->HW = c.hasher == 0 ? 5 : 7;
    int rc = 0;
    // Stages per batch: chunking (W, scalar-unit bound), SHA (A, VALU-bound), index + store (B,
    // memory-bound).  By default W is A (two stages: front = chunking + SHA, back = index + store);
    // the front is the critical path, B has slack.  HDRF_PRIO: 1 = W, A high (default), 0 = equal,
    // 2 = B high.
    int lo_prio = 0, hi_prio = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio);
    const char *pe = std::getenv("HDRF_PRIO");
    const int prio_mode = pe ? std::atoi(pe) : 1;
    // 3 = only A (SHA) high: chunking of a later batch then fills the slots SHA leaves
    const int pa = (prio_mode == 1 || prio_mode == 3) ? hi_prio : lo_prio, pb = prio_mode == 2 ? hi_prio : lo_prio;
    const int pw = prio_mode == 1 ? hi_prio : lo_prio;
    if (hipSetDevice(c.device) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->st, hipStreamNonBlocking, pa) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->stB, hipStreamNonBlocking, pb) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->stB2, hipStreamNonBlocking, pb) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->stW, hipStreamNonBlocking, pw) != hipSuccess ||
        hipStreamCreateWithPriority(&ctx->stG, hipStreamNonBlocking, pw) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stC, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stD, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stL[0], hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&ctx->stL[1], hipStreamNonBlocking) != hipSuccess) {
        free_all(ctx);
        delete ctx;
        return HDRF_E_HIP;
    }
    const int B = c.max_batch_blocks;
    ctx->max_batch = B;
    // minimum chunk is window+2 bytes; +2 for the drop-last/append rule and rounding
    ctx->cap_blk = (int)(c.max_block_bytes / (c.window + 2) + 2);
    ctx->ntiles = (ctx->cap_blk + 255) / 256;
    ctx->ev_cap = (int)(B * (c.max_block_bytes / ((int64_t)c.container_max - c.max_chunk) + 2) + 16);
    ctx->closed_cap = 3 * ctx->ev_cap;
    ctx->coll_cap = 1 << 16;
    const size_t nchunk = (size_t)B * ctx->cap_blk;
    for (auto &S : ctx->sl)
        if (!rc) rc = alloc_slot(ctx, S);
    if (!rc && ((rc = dalloc(ctx, &ctx->d_tab, (size_t)1 << c.index_log2)) ||
                (rc = dalloc(ctx, &ctx->d_arena, (size_t)c.arena_slots * c.container_max + 256)) ||
                (rc = dalloc(ctx, &ctx->d_alloc, 1)))) {
    }
    if (!rc && c.compressor == 2) {
        ctx->cslot = lz4_slot_bytes(c.container_max);
        rc = dalloc(ctx, &ctx->d_carena, (size_t)c.arena_slots * ctx->cslot + 256);
    }
    ctx->G = c.n_ranks;
    ctx->rank = c.rank;
    if (!rc && ctx->G > 1) {
        // scratch table for the batch's local aggregation: >= 1.5x the expected distinct chunks
        // (mean chunk ~949 B on random data; a table-full condition is reported, never silent)
        const double expect = 1.5 * (double)B * (double)c.max_block_bytes / 900.0;
        int lg = 16;
        while (lg < 31 && (double)(1ull << lg) < expect) lg++;
        ctx->scratch_log2 = lg;
        ctx->gx_cap = (int64_t)nchunk;
        // batches in the node-global pipeline: the fronts of the next ones (chunking on W, SHA on A,
        // local aggregation on X) run while the oldest goes through its exchanges and back phases
        const char *gd = getenv("HDRF_GX_DEPTH");
        ctx->gx_depth = std::max(2, std::min(kSlots, gd ? atoi(gd) : 3));
        ctx->fn_mcap = gx_fn_mcap(c.container_max, c.window, B);
        ctx->fn_bytes = gx_fn_bytes(c.container_max, c.window, B);
        const size_t nrec = (size_t)ctx->G * (size_t)ctx->gx_cap;
        for (int i = 0; i < ctx->gx_depth && !rc; i++)
            if ((rc = dalloc(ctx, &ctx->d_scratch[i], (size_t)1 << lg)) || (rc = dalloc(ctx, &ctx->d_gxe[i], 64)) ||
                (rc = halloc(ctx, &ctx->sl[i].h_gx, 1))) {
            }
        if (!rc && hipStreamCreateWithFlags(&ctx->stX, hipStreamNonBlocking) != hipSuccess)
            rc = set_err(ctx, HDRF_E_HIP, "hipStreamCreate failed");
        if (!rc && c.timing)
            for (auto &T : ctx->gxt)
                for (auto &e : T.ev)
                    if (!rc && hipEventCreate(&e) != hipSuccess) rc = set_err(ctx, HDRF_E_HIP, "hipEventCreate failed");
        if (rc) {
        } else if ((rc = dalloc(ctx, &ctx->d_x3want, 64)) || (rc = dalloc(ctx, &ctx->d_gxst, 4)) ||
            (rc = dalloc(ctx, &ctx->d_gx_err, 1)) ||
            (rc = dalloc(ctx, &ctx->d_gx_counts, 64)) ||
            (rc = dalloc(ctx, &ctx->d_gx_rcounts, 64)) || (rc = dalloc(ctx, &ctx->d_gx_x3exp, 64)) ||
            (rc = dalloc(ctx, &ctx->d_oslot, nrec)) ||
            (rc = dalloc(ctx, &ctx->d_oflags, nrec))) {
        }
        // owner slots start defined (hdrf_gx_owner's kernels never read a slot the claim did not write
        // once an error is raised, but a defined value keeps any later misuse inside the table)
        if (!rc && (hipMemset(ctx->d_oslot, 0, sizeof(uint32_t) * nrec) != hipSuccess ||
                    hipMemset(ctx->d_gx_err, 0, sizeof(int)) != hipSuccess))
            rc = set_err(ctx, HDRF_E_HIP, "hipMemset failed");
    }
    ctx->timing = c.timing != 0;
    ctx->fused = fused_front() && c.n_ranks <= 1;     // (node-global fronts keep the two-pass front)
    {
        int ncu = 0;
        if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, c.device) == hipSuccess && ncu > 0)
            ctx->n_cu = ncu;
    }
    if (!rc) rc = init_state(ctx, true);
    if (rc) {
        fprintf(stderr, "hdrf_open: %s\n", ctx->err.c_str());
        free_all(ctx);
        delete ctx;
        return rc;
    }
    *out = ctx;
    return 0;
}

extern "C" int hdrf_close(hdrf_ctx *ctx)
{
    if (!ctx) return HDRF_E_INVAL;
    (void)drain(ctx);
    free_all(ctx);
    delete ctx;
    return 0;
}

extern "C" const char *hdrf_last_error(const hdrf_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }
extern "C" int hdrf_digest_len(const hdrf_ctx *ctx) { return ctx ? ctx->H : HDRF_E_INVAL; }

extern "C" int hdrf_reset(hdrf_ctx *ctx)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    // a receiver may still be appending to a buffer without the lock: refuse rather than race it
    for (int i = 0; i < hdrf_ctx::kRx; i++)
        if (ctx->rx[i].state.load() == 1)
            return set_err(ctx, HDRF_E_INVAL, "a block is being received (hdrf_submit_slot or hdrf_rx_cancel first)");
    return init_state(ctx, false);
}

// A fresh DataNode without draining the pipeline (bench steps back to back, a DataNode's volume
// re-initialised while blocks are in flight): the batches already submitted complete against the
// old state; the next submit starts a new index generation (the next epoch of the tag words, so no
// table clear), the allocator is re-seeded on the index stream after the old batches' store part,
// and the host side (containers, recipes, allocator view, totals) is reset when that batch is
// completed (wait_one), after every older batch.  Single-node contexts.  Durable containers
// (retain_containers): the old generation's containers are drained as its batches complete, before
// the new generation's first batch is waited for (that wait fails otherwise: the new generation
// reuses the container ids); the slot rings continue across the generations, so no slot the old
// generation may still hand out is reopened early.
extern "C" int hdrf_reset_async(hdrf_ctx *ctx)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    for (int i = 0; i < hdrf_ctx::kRx; i++)
        if (ctx->rx[i].state.load() == 1)
            return set_err(ctx, HDRF_E_INVAL, "a block is being received (hdrf_submit_slot or hdrf_rx_cancel first)");
    if (ctx->G > 1) {
        // node-global: the switch is made by the back phases of the next launched front's batch
        // (hdrf_gx_owner: the next epoch, the node's allocator re-seeded on the back stream after the
        // old batches' commits; hdrf_gx_place_wait: the host side), since the owner phases of the
        // batches in flight are still to be enqueued with the old epoch
        if (ctx->gx_nfront == ctx->gx_nback && !ctx->gen_pending) return init_state(ctx, false);
        ctx->gen_pending = true;
        return 0;
    }
    if (ctx->nsub == ctx->nwait && !ctx->gen_pending) return init_state(ctx, false);   // nothing in flight
    ctx->gen_clear = ctx->gen_clear || ctx->epoch >= 255;
    ctx->epoch = ctx->epoch >= 255 ? 1 : ctx->epoch + 1;
    ctx->bfirst = ctx->batch + 1;
    // durable containers: the new generation continues every slot ring past the old open container
    // (idx_clear_kernel), which stays the old generation's until the switch: one more slot held per
    // switch still in flight (a second hdrf_reset_async before the first switch was waited for holds
    // a second one; calls with no submit in between make one switch)
    if (ctx->cfg.retain_containers && !ctx->gen_pending) ctx->gen_reserve++;
    ctx->gen_pending = true;
    return 0;
}

// container id -> slot bookkeeping after a batch
static void note_container(hdrf_ctx *ctx, uint32_t id, uint32_t slot, uint32_t len, int closed, uint32_t clen = 0)
{
    auto so = ctx->slot_owner.find(slot);
    if (so != ctx->slot_owner.end() && so->second != id) {
        // durable mode: the ring check in submit() keeps undrained closed containers out of reach
        if (ctx->cfg.retain_containers)
            for (uint32_t u : ctx->pend_closed)
                if (u == so->second) ctx->lost = true;
        ctx->containers.erase(so->second);
    }
    ctx->slot_owner[slot] = id;
    ctx->containers[id] = ContainerInfo{slot, len, closed, clen};
}

static ChunkScratch chunk_scratch(Slot &S, int compressor = 1)
{
    ChunkScratch X;
    X.ring = compressor == 2 ? 0 : 1;
    X.gm = S.d_gm; X.gstride = S.gstride; X.rq = S.d_rq; X.rq_count = S.d_rq_count; X.rq_cap = (int)S.meta_cap;
    X.rqkeep = S.d_rqkeep;
    X.irr = S.d_irr; X.path = S.d_path; X.jx = S.d_jx; X.jt = S.d_jt; X.jcap = S.jcap; X.wgsum = S.d_wgsum;
    X.maxw = S.maxw_cap;
    return X;
}

// HDRF_FUSED=1: the front cuts and hashes in one pass over the bytes (lanehash.hip) instead of the
// granule pass + lane walk (chunk.hip) followed by the SHA lanes (sha.hip); single-node contexts.
// Read when a context opens, so a process may hold contexts of both kinds (the tests do).
static bool fused_front()
{
    const char *e = getenv("HDRF_FUSED");
    return e && atoi(e) != 0;
}

// Validate a batch and fill the slot's (pinned) descriptors: the lane segmentation of the chunking
// pass (chunk.hip).  seg_len = segment_bytes / 63 rounded down to a multiple of window + 2, within
// [4, 20] x 702 B.  Grows the slot's speculative lists when needed (the slot's previous batch has
// completed).
static int prepare_blocks(hdrf_ctx *ctx, Slot &S, int32_t nblocks, const uint8_t *const *dev_data,
                          const uint64_t *len, const uint64_t *readable)
{
    if (nblocks < 1 || nblocks > ctx->max_batch || !dev_data || !len || !readable)
        return set_err(ctx, HDRF_E_INVAL, "bad batch arguments");
    const hdrf_cfg &c = ctx->cfg;
    int64_t total = 0, max_len = 0;
    for (int b = 0; b < nblocks; b++) {
        if ((int64_t)len[b] > c.max_block_bytes) return set_err(ctx, HDRF_E_INVAL, "block larger than max_block_bytes");
        if (readable[b] < len[b] + kSlack) return set_err(ctx, HDRF_E_INVAL, "readable must be >= len + 64");
        if (((uintptr_t)dev_data[b] & 15) != 0) return set_err(ctx, HDRF_E_INVAL, "block data must be 16-B aligned");
        total += (int64_t)len[b];
        max_len = std::max(max_len, (int64_t)len[b]);
    }
    S.max_len = max_len;
    const int unit = c.window + 2;
    // one lane per segment: a block of any size has thousands of lanes, so the segment length
    // follows segment_bytes alone (shorter segments only raise the share of boundaries whose
    // chains have not met within the next segment, which then take the repair pass)
    int wins = std::max(kSegMinWin, std::min(kSegMaxWin, (int)(c.segment_bytes / kWaveSegs / unit)));
    // HDRF_SEG_WINS (A/B): the two-pass front's segment length in windows, over segment_bytes
    static const int wins_env = [] { const char *e = getenv("HDRF_SEG_WINS"); return e ? atoi(e) : 0; }();
    if (wins_env > 0 && !ctx->fused) wins = std::max(kSegMinWin, std::min(kSegMaxWin, wins_env));
    if (ctx->fused) {
        // the fused pass (lanehash.hip): every lane does the same work (its segment, 64 B per step),
        // so a second, partial round of waves costs as much as a full one — the shortest segments
        // whose waves fit one round (16 per CU at its 99 VGPRs; 4 GiB batch: 24 windows, 4064 waves)
        const int64_t cap_waves = (int64_t)ctx->n_cu * 16;
        auto waves_for = [&](int wn) {
            int64_t wv = 0;
            for (int b = 0; b < nblocks; b++) {
                const int64_t ns = std::max<int64_t>(1, ((int64_t)len[b] + (int64_t)wn * unit - 1) / ((int64_t)wn * unit));
                wv += (ns + kWaveSegs - 1) / kWaveSegs;
            }
            return wv;
        };
        wins = kSegMinWin;
        while (wins < kSegMaxWinF && waves_for(wins) > cap_waves) wins++;
    }
    (void)total;
    const int seg_len = wins * unit;
    int seg0 = 0, wave0 = 0;
    for (int b = 0; b < nblocks; b++) {
        BlockDesc &d = S.h_desc[b];
        d.data = dev_data[b];
        d.len = len[b];
        d.readable = readable[b];
        d.nseg = (int)std::max<int64_t>(1, ((int64_t)len[b] + seg_len - 1) / seg_len);
        d.seg_len = seg_len;
        d.seg0 = seg0;
        d.wave0 = wave0;
        seg0 += d.nseg;
        wave0 += (d.nseg + kWaveSegs - 1) / kWaveSegs;
    }
    S.total_waves = wave0;
    S.total_segs = seg0;
    int max_nseg = 1;
    for (int b = 0; b < nblocks; b++) max_nseg = std::max(max_nseg, S.h_desc[b].nseg);
    S.max_nseg = max_nseg;
    const int maxw = (max_nseg + 255) / 256;
    if (maxw > S.maxw_cap) {
        (void)hipFree(S.d_wgsum);
        S.d_wgsum = nullptr;
        S.maxw_cap = 0;
        if (int rc = dalloc(ctx, &S.d_wgsum, (size_t)ctx->max_batch * maxw)) return rc;
        S.maxw_cap = maxw;
    }
    S.spec_cap = lane_spec_cap(seg_len, c.window);
    const size_t words = (size_t)seg0 * S.spec_cap;
    if ((size_t)seg0 > S.meta_cap) {
        (void)hipFree(S.d_meta);
        (void)hipFree(S.d_rq);
        S.d_meta = nullptr;
        S.d_rq = nullptr;
        S.meta_cap = 0;
        if (int rc = dalloc(ctx, &S.d_meta, (size_t)seg0)) return rc;
        if (int rc = dalloc(ctx, &S.d_rq, (size_t)seg0)) return rc;
        (void)hipFree(S.d_irr);
        S.d_irr = nullptr;
        if (int rc = dalloc(ctx, &S.d_irr, (size_t)seg0 / 32 + 2)) return rc;
        S.meta_cap = (size_t)seg0;
    }
    if (words > S.spec_words) {
        (void)hipFree(S.d_spec);
        S.d_spec = nullptr;
        S.spec_words = 0;
        if (int rc = dalloc(ctx, &S.d_spec, words)) return rc;
        S.spec_words = words;
    }
    if (ctx->fused) {
        if (!S.d_need)
            if (int rc = dalloc(ctx, &S.d_need, (size_t)ctx->max_batch * ctx->cap_blk)) return rc;
        if (!S.d_nlist)
            if (int rc = dalloc(ctx, &S.d_nlist, (size_t)ctx->max_batch * ctx->cap_blk)) return rc;
        if (!S.d_gmneed)
            if (int rc = dalloc(ctx, &S.d_gmneed, (size_t)ctx->max_batch)) return rc;
        if (words * ctx->HW > S.sdig_words) {
            (void)hipFree(S.d_sdig);
            S.d_sdig = nullptr;
            S.sdig_words = 0;
            if (int rc = dalloc(ctx, &S.d_sdig, words * ctx->HW)) return rc;
            S.sdig_words = words * ctx->HW;
        }
        if ((size_t)seg0 + 1 > S.bdig_segs) {
            (void)hipFree(S.d_bdig);
            S.d_bdig = nullptr;
            S.bdig_segs = 0;
            if (int rc = dalloc(ctx, &S.d_bdig, ((size_t)seg0 + 1) * ctx->HW)) return rc;
            S.bdig_segs = (size_t)seg0 + 1;
        }
    }
    return 0;
}

static StoreParams store_params(const hdrf_ctx *ctx, int nblocks)
{
    const hdrf_cfg &c = ctx->cfg;
    StoreParams P;
    P.nblocks = nblocks; P.cap_blk = ctx->cap_blk; P.ntiles = ctx->ntiles;
    P.n_thread = c.n_thread; P.min_mt = c.min_mt_chunks; P.cmax = c.container_max;
    P.nslots = (uint32_t)c.arena_slots; P.ev_cap = ctx->ev_cap; P.closed_cap = ctx->closed_cap;
    return P;
}

static float elapsed(hipEvent_t a, hipEvent_t b)
{
    float ms = 0;
    return hipEventElapsedTime(&ms, a, b) == hipSuccess ? ms : 0.f;
}

// Upper bound on the containers one storer range can close in a batch of `bytes` new bytes: a
// container closes when its length plus the next chunk exceeds container_max, so it holds more
// than container_max - max_chunk - 1 bytes, and two consecutive closes hold more than
// container_max between them (DN/DataDeduplicator.java:748-796).
static uint32_t close_bound(const hdrf_cfg &c, uint64_t bytes)
{
    const uint64_t a = bytes / std::max<uint64_t>(1, (uint64_t)c.container_max - (uint64_t)c.max_chunk - 1);
    const uint64_t b = 2 * bytes / c.container_max;
    return (uint32_t)std::min<uint64_t>(std::min(a, b), 1u << 30) + 1;
}

// Enqueue one batch: front on stream A, back on stream B (see the file comment).
static int submit(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                  const uint64_t *readable, const uint64_t *block_ids, bool after_copy = false)
{
    if (ctx->nsub - ctx->nwait >= (uint64_t)kSlots)
        if (int rc = wait_one(ctx)) return rc;
    Slot &S = ctx->sl[ctx->nsub % kSlots];
    const hdrf_cfg &c = ctx->cfg;
    if (int rc = prepare_blocks(ctx, S, nblocks, dev_data, len, readable)) return rc;
    S.close_bound = 0;
    if (c.retain_containers) {
        // durable containers: the ring of every storer range (arena_slots / 4 slots, its open
        // container included) must keep room for the closes this batch and the batches in flight
        // can make without reaching an undrained closed container
        uint64_t bytes = 0;
        for (int b = 0; b < nblocks; b++) bytes += len[b];
        const uint32_t bound = close_bound(c, bytes), per = (uint32_t)(c.arena_slots / 4);
        // Only completed batches' containers can be drained: when the batches in flight are part of
        // what fills the ring, the recovery is hdrf_wait_batch (oldest), then hdrf_drain_containers,
        // then the submit again; the message names the step.
        for (int t = 0; t < c.n_thread; t++)
            if ((uint64_t)ctx->undrained[t] + ctx->inflight_bound + ctx->gen_reserve + bound > per - 1)
                return set_err(ctx, HDRF_E_CAPACITY,
                               "container arena: the ring of storer range " + std::to_string(t) + " is full (" +
                                   std::to_string(ctx->undrained[t]) + " undrained closed containers, " +
                                   std::to_string(ctx->inflight_bound) + " closes bounded for batches in flight)" +
                                   (ctx->inflight_bound ? " (hdrf_wait_batch, then hdrf_drain_containers)"
                                                        : " (hdrf_drain_containers first)"));
        S.close_bound = bound;
        ctx->inflight_bound += bound;
    }
    S.ids.assign(nblocks, 0);
    if (block_ids) S.ids.assign(block_ids, block_ids + nblocks);
    S.lens.assign(len, len + nblocks);
    S.nblocks = nblocks;
    S.gen_reset = ctx->gen_pending;                   // the first batch of a fresh generation (hdrf_reset_async)
    ctx->gen_pending = false;
    const uint32_t cur = ++ctx->batch;
    // chunking runs on its own stream W (HDRF_STREAMS=2: shares stream A with SHA).  Measured with
    // the two-pass lane walker (r02): three streams 992 GB/s vs two 919 — the walk's latency-bound
    // kernels and the HBM-bound granule pass overlap SHA's VALU stream of the previous batch
    static const int nstreams = [] { const char *e = getenv("HDRF_STREAMS"); return e ? atoi(e) : 3; }();
    hipStream_t W = nstreams == 3 ? ctx->stW : ctx->st, A = ctx->st, Bst = ctx->stB;
    // HDRF_GMAX_STREAM=1: the granule-max pass on stream G, so the next batch's (HBM-bound) pass
    // runs while W walks and stitches this one (latency-bound)
    static const bool gstream = [] { const char *e = getenv("HDRF_GMAX_STREAM"); return e && atoi(e) != 0; }();
    hipStream_t G = gstream ? ctx->stG : W;
    // ---- chunking on W: the slot's previous batch has completed (wait_one ran), so W may overwrite it
    if (after_copy) HIPCK(hipStreamWaitEvent(G, S.copy_done, 0));
    HIPCK(hipMemcpyAsync(S.d_blocks, S.h_desc, sizeof(BlockDesc) * nblocks, hipMemcpyHostToDevice, G));
    Marker mw;
    mw.ev = ctx->timing ? S.evW : nullptr;
    // (the fused front writes d_dig on W: after the recipe copies of the slot's previous batch read it)
    const bool fz_on = ctx->fused;
    if (fz_on && S.recipe_pending) HIPCK(hipStreamWaitEvent(W, S.recipe_done, 0));
    const FusedFront fz{c.hasher, S.d_sdig, S.d_bdig, S.d_dig, S.d_need, S.d_gmneed};
    HIPCK(launch_chunking(S.d_blocks, nblocks, S.max_len, S.max_nseg, S.total_waves, S.total_segs,
                          chunk_scratch(S, c.compressor), c.window, c.max_chunk, S.d_spec, S.spec_cap, S.d_meta, S.d_bst,
                          S.d_off, ctx->cap_blk, S.d_err, W, &mw, G, S.gmax_done, fz_on ? &fz : nullptr));
    mw.mark(W);
    HIPCK(hipEventRecord(S.walk_done, W));
    // ---- fingerprints on A (after the recipe copies of the slot's previous batch read d_dig); the fused
    // front leaves only the chunks marked in d_need (each block's last one, repairs, fallbacks)
    HIPCK(hipStreamWaitEvent(A, S.walk_done, 0));
    if (S.recipe_pending) HIPCK(hipStreamWaitEvent(A, S.recipe_done, 0));
    Marker ma;
    ma.ev = ctx->timing ? S.evA : nullptr;
    if (fz_on)
        HIPCK(launch_sha_need(c.hasher, S.d_blocks, nblocks, S.d_off, S.d_bst, ctx->cap_blk, S.d_dig, S.d_queue, S.d_need,
                              S.d_nlist, A, &ma));
    else
        HIPCK(launch_sha(c.hasher, S.d_blocks, nblocks, S.d_off, S.d_bst, ctx->cap_blk, S.d_dig, S.d_queue, ctx->sha_long, A,
                         &ma));
    ma.mark(A);
    HIPCK(hipEventRecord(S.front_done, A));
    // ---- back, index part, in block order on stream B: claim .. decide, then idx_finalize takes the
    // batch-local state out of the index (designated chunks, block counts, entries cleared), so the
    // next batch's index part may run while this batch is stored on stream B2
    HIPCK(hipStreamWaitEvent(Bst, S.front_done, 0));
    if (S.gen_reset) {
        // a fresh generation: the old batches' store part (stream B2: place writes index values, the
        // flush walk the allocator) is finished before this index part claims entries of the new epoch;
        // then the allocator is re-seeded (and the table cleared when the epoch wrapped)
        if (ctx->nsub > ctx->nwait) HIPCK(hipStreamWaitEvent(Bst, ctx->sl[(ctx->nsub - 1) % kSlots].back_done, 0));
        HIPCK(launch_index_clear(ctx->d_tab, ctx->gen_clear ? c.index_log2 : -1, ctx->d_alloc, initial_alloc(ctx), Bst,
                                 c.retain_containers ? (uint32_t)(c.arena_slots / 4) : 0u));
        ctx->gen_clear = false;
    }
    // HDRF_DECIDE_DESIG=0 (A/B): idx_finalize reads every designated entry (round-3 c2 behaviour)
    static const bool decide_desig = [] { const char *e = getenv("HDRF_DECIDE_DESIG"); return !e || atoi(e) != 0; }();
    Marker mb;
    mb.ev = ctx->timing ? S.evB : nullptr;
    HIPCK(launch_index(c.hasher, S.d_bst, nblocks, ctx->cap_blk, S.d_off, S.d_dig, ctx->d_tab, c.index_log2, cur,
                       ctx->bfirst, tag_mask(ctx), S.d_slot, S.d_coll, S.d_ncoll, ctx->coll_cap, S.d_flags, S.d_tilesum, ctx->ntiles,
                       S.d_err, Bst, &mb, decide_desig ? S.d_dcnt : nullptr));
    HIPCK(launch_index_finalize(S.d_bst, nblocks, ctx->cap_blk, ctx->ntiles, ctx->d_tab, S.d_slot, S.d_flags, S.d_dcnt,
                                Bst));
    if (ctx->timing) HIPCK(hipEventRecord(S.evB[9], Bst));
    HIPCK(hipEventRecord(S.idx_done, Bst));
    // ---- back, store part, in block order on stream B2 (scans, flush walk, place, read-back)
    // HDRF_SPLIT_B=0: the store part on stream B too (A/B of the split)
    static const bool split_b = [] { const char *e = getenv("HDRF_SPLIT_B"); return !e || atoi(e) != 0; }();
    hipStream_t B2 = split_b ? ctx->stB2 : Bst;
    HIPCK(hipStreamWaitEvent(B2, S.idx_done, 0));
    HIPCK(hipMemsetAsync(S.d_nclosed, 0, sizeof(uint32_t), B2));
    StoreParams P = store_params(ctx, nblocks);
    // When batches are pipelined (one already in flight), this batch's place kernel overlaps the
    // next batch's front stage (the critical path): a dynamic-LDS reservation caps place at one
    // wave per SIMD so SHA keeps its wave slots (measured +1.5-2% on the config-2 bench; alone,
    // place wants full occupancy).  Under compressor 2 the reservation is 16 KiB: place then fits on
    // a CU as soon as one LZ4 wave of a draining pass leaves it (config 4: 36.96 / 37.01 vs 35.92 /
    // 35.91 GB/s with 40 KiB; 24 KiB 36.5, 9 KiB 36.4; profiles/r02_c4_place_ab.txt).  Round 5, after
    // the LZ4 parse got shorter: 8 KiB 47.31 / 47.27 vs 16 KiB 47.13 / 47.10, 24 KiB 46.68 / 46.74
    // (profiles/r05_c4knobs_ab.txt), so 8 KiB.  HDRF_PLACE_LDS overrides the reservation (bytes).
    static const int place_lds_env = [] { const char *e = getenv("HDRF_PLACE_LDS"); return e ? atoi(e) : -1; }();
    const int place_lds = place_lds_env >= 0 ? place_lds_env : (c.compressor == 2 ? 8192 : 40960);
    if (ctx->nsub > ctx->nwait) P.place_lds = place_lds;
    // HDRF_PLACE_DEEP=1: the place copy keeps four 16-B words per thread in flight instead of two
    static const int place_deep_env = [] { const char *e = getenv("HDRF_PLACE_DEEP"); return e ? atoi(e) : 0; }();
    P.place_deep = place_deep_env;
    if (c.compressor == 2) {
        // The compression of earlier batches runs on the LZ4 streams, off stream B, so batch k+1's
        // index and store overlap batch k's LZ4 and the LZ4 passes of consecutive batches overlap
        // each other (no per-batch tail on the critical chain).  A place kernel may reopen an arena
        // slot only after the LZ4 pass reading it finished: a slot closed in batch j is reopened
        // at the (arena_slots/4)-th open of its ring after it, and a batch opens at most as many
        // containers per range as it closes (close_bound), so stream B waits for an in-flight
        // batch's LZ4 only when the closes bound from it up to this batch could wrap the ring.
        uint64_t bytes = 0;
        for (int b = 0; b < nblocks; b++) bytes += len[b];
        S.lz_bound = close_bound(c, bytes);
        const uint64_t per = (uint64_t)(c.arena_slots / 4);
        uint64_t sum = S.lz_bound;
        for (uint64_t j = ctx->nsub - 1; j + 1 > ctx->nwait; j--) {   // in flight, newest first
            const Slot &Pj = ctx->sl[j % kSlots];
            sum += Pj.lz_bound;
            // (a fresh generation restarts every ring at its first slot: every pass in flight first)
            if (sum + 1 >= per || S.gen_reset) HIPCK(hipStreamWaitEvent(B2, Pj.lz_done, 0));
            if (j == 0) break;
        }
    }
    HIPCK(launch_store(P, S.d_blocks, S.d_bst, S.d_off, S.d_flags, S.d_tilesum, S.d_tilepre, S.d_store, S.d_pre,
                       ctx->d_alloc, S.d_rstate, S.d_ev, S.d_closed, S.d_nclosed, S.d_slot, ctx->d_tab, ctx->d_arena,
                       S.d_pcid, S.d_ppos, S.d_err, B2, &mb, nullptr, S.d_dcnt));
    if (c.compressor == 2) {    // compression stage: closed containers -> Lz4Codec files (:770-779)
        hipStream_t L = ctx->stL[cur & 1];
        HIPCK(hipEventRecord(S.placed, B2));
        HIPCK(hipStreamWaitEvent(L, S.placed, 0));
        HIPCK(launch_lz4(S.d_closed, S.d_nclosed, ctx->closed_cap, c.container_max, ctx->d_arena, ctx->d_carena,
                         ctx->cslot, S.d_segclen, S.d_filelen, S.d_lzwork, L));
        mb.mark(L);
        HIPCK(hipMemcpyAsync(S.h_filelen, S.d_filelen, sizeof(uint32_t) * ctx->closed_cap, hipMemcpyDeviceToHost, L));
        HIPCK(hipEventRecord(S.lz_done, L));
    } else {
        mb.mark(B2);
    }
    HIPCK(hipMemcpyAsync(S.h_bst, S.d_bst, sizeof(BlockState) * nblocks, hipMemcpyDeviceToHost, B2));
    HIPCK(hipMemcpyAsync(S.h_store, S.d_store, sizeof(uint64_t) * nblocks, hipMemcpyDeviceToHost, B2));
    HIPCK(hipMemcpyAsync(S.h_alloc, ctx->d_alloc, sizeof(AllocState), hipMemcpyDeviceToHost, B2));
    HIPCK(hipMemcpyAsync(S.h_err, S.d_err, sizeof(int), hipMemcpyDeviceToHost, B2));
    HIPCK(hipMemcpyAsync(S.h_nclosed, S.d_nclosed, sizeof(uint32_t), hipMemcpyDeviceToHost, B2));
    HIPCK(hipMemcpyAsync(S.h_long, S.d_queue + 64, sizeof(uint32_t), hipMemcpyDeviceToHost, B2));
    HIPCK(hipMemcpyAsync(S.h_closed, S.d_closed, sizeof(ClosedRec) * ctx->closed_cap, hipMemcpyDeviceToHost, B2));
    HIPCK(hipEventRecord(S.back_done, B2));
    S.pending = true;
    ctx->nsub++;
    return 0;
}

static int complete_state(hdrf_ctx *ctx, Slot &S);

// space for one recipe's digests in the device recipe store (4-B aligned words; entries start
// on 16 B)
static int recipe_alloc(hdrf_ctx *ctx, uint64_t bytes, uint32_t key, uint32_t n, uint8_t **dst)
{
    constexpr uint64_t kChunk = 256ull << 20;
    if (bytes > kChunk) return set_err(ctx, HDRF_E_CAPACITY, "recipe larger than a recipe-store chunk");
    if (ctx->rcur < ctx->rchunks.size() && ctx->rhead + bytes > kChunk) { ctx->rcur++; ctx->rhead = 0; }
    if (ctx->rcur >= ctx->rchunks.size()) {
        uint8_t *p = nullptr;
        HIPCK(hipMalloc((void **)&p, kChunk));
        ctx->rchunks.push_back(p);
        ctx->rcur = (uint32_t)ctx->rchunks.size() - 1;
        ctx->rhead = 0;
    }
    *dst = ctx->rchunks[ctx->rcur] + ctx->rhead;
    ctx->recipes[key] = hdrf_ctx::RecipeLoc{ctx->rcur, ctx->rhead, n};
    ctx->rhead += (bytes + 15) & ~15ull;
    return 0;
}

// GET longToBytes(id,4): [BE32 size | digests] out of the device store; the caller drained.
// 1 found, 0 absent, < 0 error
static int fetch_recipe(hdrf_ctx *ctx, uint32_t key, std::vector<uint8_t> &r)
{
    auto it = ctx->recipes.find(key);
    if (it == ctx->recipes.end()) return 0;
    const int64_t ln = ctx->lengths[key];
    r.resize(4 + (size_t)it->second.n * ctx->H);
    r[0] = (uint8_t)(ln >> 24); r[1] = (uint8_t)(ln >> 16); r[2] = (uint8_t)(ln >> 8); r[3] = (uint8_t)ln;
    if (it->second.n)
        HIPCK(hipMemcpy(r.data() + 4, ctx->rchunks[it->second.chunk] + it->second.off, (size_t)it->second.n * ctx->H,
                        hipMemcpyDeviceToHost));
    return 1;
}

// After a batch's read-back landed: container / recipe / allocator bookkeeping.
static int complete_slot(hdrf_ctx *ctx, int si, bool timed)
{
    Slot &S = ctx->sl[si];
    const int nblocks = S.nblocks;
    if (ctx->timing && timed) {
        ctx->stage_ms[11] += elapsed(S.evW[0], S.evW[1]);
        for (int i = 0; i < 2; i++) ctx->stage_ms[i] += elapsed(S.evW[i + 1], S.evW[i + 2]);
        for (int i = 0; i < 2; i++) ctx->stage_ms[2 + i] += elapsed(S.evA[i], S.evA[i + 1]);
        // (evB[9]: the end of the index part on stream B; evB[3..]: the store part on stream B2)
        for (int i = 0; i < 6; i++) ctx->stage_ms[4 + i] += elapsed(S.evB[i], i == 2 ? S.evB[9] : S.evB[i + 1]);
        ctx->stage_ms[10] += elapsed(S.evB[7], S.evB[8]);
    }
    ctx->res = si;
    ctx->last_nblocks = nblocks;
    ctx->h_alloc = *S.h_alloc;
    const int herr = *S.h_err;
    if (herr) {
        HIPCK(hipMemsetAsync(S.d_err, 0, sizeof(int), ctx->stB));
        HIPCK(hipStreamSynchronize(ctx->stB));
        *S.h_err = 0;
        return device_error(ctx, herr);
    }
    return complete_state(ctx, S);
}
static int complete_state(hdrf_ctx *ctx, Slot &S)
{
    const hdrf_cfg &c = ctx->cfg;
    const int nblocks = S.nblocks;
    const uint32_t nclosed = *S.h_nclosed;
    ctx->sha_long = *S.h_long != 0;               // long SHA lanes for the next submissions
    if ((int)nclosed > ctx->closed_cap) return set_err(ctx, HDRF_E_CAPACITY, "closed-container list overflow");
    ctx->inflight_bound -= std::min(ctx->inflight_bound, S.close_bound);
    S.close_bound = 0;
    for (uint32_t i = 0; i < nclosed; i++) {
        const ClosedRec &r = S.h_closed[i];
        // (node-global contexts compress after the head pieces are gathered: hdrf_gx_compress)
        const uint32_t flen = c.compressor == 2 && ctx->G == 1 ? S.h_filelen[i] : r.len;
        note_container(ctx, r.id, r.slot, r.len, 1, flen);
        if (c.retain_containers) {
            ctx->pend_closed.push_back(r.id);
            ctx->undrained[std::min<uint32_t>(r.id >> 22, 3)]++;
        }
        ctx->stats.closed_containers++;
        ctx->stats.closed_raw_bytes += r.len;
        ctx->stats.closed_file_bytes += flen;
    }
    for (int t = 0; t < c.n_thread; t++)
        if (ctx->h_alloc.exists[t]) note_container(ctx, ctx->h_alloc.id[t], ctx->h_alloc.slot[t], ctx->h_alloc.cur[t], 0);
    if (ctx->lost) return set_err(ctx, HDRF_E_CAPACITY, "an undrained closed container's arena slot was reused");
    ctx->have_alloc = 1;                              // storeDB always SETs "blockID" (:389)
    for (int b = 0; b < nblocks; b++) {
        ctx->stats.blocks++;
        ctx->stats.logical_bytes += S.lens[b];
        ctx->stats.new_bytes += S.h_store[b];
        ctx->stats.chunks += S.h_bst[b].n_chunks;
        ctx->stats.recipe_bytes += 4 + (uint64_t)S.h_bst[b].n_chunks * ctx->H;
    }
    ctx->stats.open_bytes = 0;
    for (int t = 0; t < c.n_thread; t++)
        if (ctx->h_alloc.exists[t]) ctx->stats.open_bytes += ctx->h_alloc.cur[t];
    // recipes (SET longToBytes(id,4) -> BE32 size | digests): the block's digests are copied on
    // the device into the recipe store off stream B (the critical chain): on stream C, or on stream R
    // once host batches put H2D copies on C (a recipe kernel there held back the copies queued behind
    // it).  R exists only then: one more stream from the open on changed how the hardware queues are
    // shared and config 4's two LZ4 passes stopped overlapping (40.5 -> 34.2 GB/s,
    // profiles/r04_c4_stream_ab.txt).  The slot's next SHA waits for the copies.
    int nj = 0;
    for (int b = 0; b < nblocks; b++) {
        const uint32_t key = (uint32_t)S.ids[b];
        ctx->lengths[key] = (int64_t)S.lens[b];
        if (c.keep_recipes) {
            const uint32_t n = (uint32_t)S.h_bst[b].n_chunks;
            uint8_t *dst = nullptr;
            if (int rc = recipe_alloc(ctx, (uint64_t)n * ctx->H, key, n, &dst)) return rc;
            S.h_rjobs[nj++] = RecipeCopy{(uint64_t)(uintptr_t)(S.d_dig + (size_t)b * ctx->cap_blk * ctx->HW),
                                         (uint64_t)(uintptr_t)dst, n * (uint32_t)ctx->HW, 0};
        }
    }
    if (nj) {
        if (ctx->host_copies && !ctx->stR) HIPCK(hipStreamCreateWithFlags(&ctx->stR, hipStreamNonBlocking));
        hipStream_t rs = ctx->host_copies ? ctx->stR : ctx->stC;
        HIPCK(hipMemcpyAsync(S.d_rjobs, S.h_rjobs, sizeof(RecipeCopy) * nj, hipMemcpyHostToDevice, rs));
        HIPCK(launch_recipe_copy(S.d_rjobs, nj, rs));
        HIPCK(hipEventRecord(S.recipe_done, rs));
        S.recipe_pending = true;
    }
    return 0;
}


// Durable containers: is any container of the current host generation not yet handed out (closed
// ones, and the bytes of the open ones)?  A new generation reuses their ids.
static bool gen_undrained(const hdrf_ctx *ctx)
{
    if (!ctx->pend_closed.empty()) return true;
    for (int t = 0; t < ctx->cfg.n_thread && ctx->have_alloc; t++) {
        if (!ctx->h_alloc.exists[t]) continue;
        auto it = ctx->containers.find(ctx->h_alloc.id[t]);
        auto h = ctx->handed.find(ctx->h_alloc.id[t]);
        const int64_t done = h != ctx->handed.end() ? h->second : 0;
        if (it != ctx->containers.end() && (int64_t)it->second.len > done) return true;
    }
    return false;
}

// Complete the oldest batch in flight (its slot is reusable once this returns).  The first batch of
// a fresh generation (hdrf_reset_async) on a durable context is refused while the old generation's
// containers are not drained, and stays in flight: hdrf_drain_containers, then hdrf_wait_batch again.
// force (drain(): a view, a reset or close): it completes anyway and the context is marked lost.
static int wait_one(hdrf_ctx *ctx, bool force)
{
    if (ctx->nwait >= ctx->nsub) return set_err(ctx, HDRF_E_INVAL, "no batch in flight");
    const int si = (int)(ctx->nwait % kSlots);
    Slot &S = ctx->sl[si];
    const bool refused = S.gen_reset && ctx->cfg.retain_containers && gen_undrained(ctx);
    if (refused && !force)
        return set_err(ctx, HDRF_E_INVAL, "hdrf_reset_async: the previous generation's containers were not "
                                          "drained before its successor's first batch was waited for "
                                          "(hdrf_drain_containers, then hdrf_wait_batch again)");
    ctx->nwait++;
    S.pending = false;
    HIPCK(hipEventSynchronize(S.back_done));
    if (ctx->cfg.compressor == 2) HIPCK(hipEventSynchronize(S.lz_done));
    for (int i = 0; i < hdrf_ctx::kRx; i++)            // its receive buffers are free again
        if (S.rx_release >> i & 1) {
            ctx->rx[i].state = 0;
            ctx->rx[i].len = 0;
        }
    S.rx_release = 0;
    if (S.gen_reset) {                                   // the first batch of a fresh generation
        if (ctx->cfg.retain_containers) {
            ctx->handed.clear();
            // this switch's ring continuation is over (one per pending durable generation switch)
            ctx->gen_reserve -= std::min<uint32_t>(ctx->gen_reserve, 1u);
        }
        reset_host(ctx);
        S.gen_reset = false;
        if (refused) {
            ctx->lost = true;
            (void)complete_slot(ctx, si, true);
            return set_err(ctx, HDRF_E_CAPACITY, "hdrf_reset_async: the previous generation's undrained containers "
                                                 "were dropped (the context needs hdrf_reset)");
        }
    }
    return complete_slot(ctx, si, true);
}

// ---- packet-granular receive (DN/BlockReceiver.java:877-896: each packet appended to bf1 as it
// arrives; :1258-1261 the finished block handed to the reducer) ------------------------------
// A packet is copied into the receive buffer's current pinned 4 MiB staging chunk (the caller may
// reuse the packet when the call returns); every full chunk goes H2D on stream C into the block's
// device buffer, overlapping the next packets and the kernels of the blocks in flight.  The two
// chunks alternate, waiting (host side) for a chunk's copy only before refilling it.  The packets
// of one block come from one receiver thread (the reference's BlockReceiver), so appends take
// only that buffer's state, not the context lock: receivers of different blocks copy in parallel.
// (touches only the receive buffer and stream C, so it runs without the context lock; the caller
// records an error under the lock)
static hipStream_t rx_stream(hdrf_ctx *ctx, const hdrf_ctx::Rx &r) { return r.st ? r.st : ctx->stC; }

// Packet bytes into the pinned staging chunk with non-temporal 16-B stores: the receiver thread does
// not read the destination lines first (a plain copy of a 64 KiB packet fetches them for ownership)
// and leaves nothing dirty in its caches for the copy engine's reads.  HDRF_RX_NT=0: std::memcpy.
static void copy_nt(uint8_t *dst, const uint8_t *src, uint64_t n)
{
    typedef long long v2 __attribute__((vector_size(16)));
    uint64_t head = (16 - ((uintptr_t)dst & 15)) & 15;
    if (head > n) head = n;
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    const uint64_t n64 = n >> 6;
    for (uint64_t i = 0; i < n64; i++) {
        v2 a, b, c, d;
        std::memcpy(&a, src + 64 * i, 16);
        std::memcpy(&b, src + 64 * i + 16, 16);
        std::memcpy(&c, src + 64 * i + 32, 16);
        std::memcpy(&d, src + 64 * i + 48, 16);
        __builtin_nontemporal_store(a, (v2 *)(dst + 64 * i));
        __builtin_nontemporal_store(b, (v2 *)(dst + 64 * i + 16));
        __builtin_nontemporal_store(c, (v2 *)(dst + 64 * i + 32));
        __builtin_nontemporal_store(d, (v2 *)(dst + 64 * i + 48));
    }
    std::memcpy(dst + 64 * n64, src + 64 * n64, n & 63);
    // Non-temporal stores are weakly ordered: fence them here, on the thread that wrote them, so
    // the staged bytes are visible before any later store of this thread (the hand-off of the block
    // to another thread that queues its last chunk's copy, e.g. hdrf_submit_slots from a submitter).
#if !defined(__HIP_DEVICE_COMPILE__)
    __builtin_ia32_sfence();
#endif
}

static bool rx_nt()
{
    static const bool on = [] { const char *e = getenv("HDRF_RX_NT"); return !e || atoi(e) != 0; }();
    return on;
}

static hipError_t rx_flush(hdrf_ctx *ctx, hdrf_ctx::Rx &r)
{
    if (r.fill == 0) return hipSuccess;
    const int c = r.cur;
    // the chunk's non-temporal stores are globally visible before the copy engine is told to read it
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipError_t e = hipMemcpyAsync(r.d + r.dst, r.h + (uint64_t)c * ctx->kRingChunk, r.fill, hipMemcpyHostToDevice,
                                  rx_stream(ctx, r));
    if (e == hipSuccess) e = hipEventRecord(r.ev[c], rx_stream(ctx, r));
    if (e != hipSuccess) return e;
    r.busy[c] = true;
    r.cur = c ^ 1;
    r.fill = 0;
    if (r.busy[r.cur]) {                               // refilling that chunk: its copy must have landed
        if ((e = hipEventSynchronize(r.ev[r.cur])) != hipSuccess) return e;
        r.busy[r.cur] = false;
    }
    return hipSuccess;
}

extern "C" int hdrf_rx_begin(hdrf_ctx *ctx, uint64_t block_id, int32_t *rx)
{
    HDRF_LOCK(ctx);
    if (!ctx || !rx) return HDRF_E_INVAL;
    if (ctx->G > 1) return set_err(ctx, HDRF_E_INVAL, "node-global context: use the hdrf_gx_* phases");
    for (int i = 0; i < hdrf_ctx::kRx; i++) {
        hdrf_ctx::Rx &r = ctx->rx[i];
        if (r.state.load() != 0) continue;
        if (!r.d) HIPCK(hipMalloc((void **)&r.d, (uint64_t)ctx->cfg.max_block_bytes + kSlack + 256));
        if (!r.h) {
            HIPCK(hipHostMalloc((void **)&r.h, 2 * ctx->kRingChunk));
            for (auto &e : r.ev) HIPCK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            static const bool own = [] { const char *e = getenv("HDRF_RX_STREAMS"); return e && atoi(e) != 0; }();
            if (own) {
                HIPCK(hipStreamCreateWithFlags(&r.st, hipStreamNonBlocking));
                HIPCK(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
            }
        }
        r.len = 0;
        r.fill = 0;
        r.dst = 0;
        r.id = block_id;
        r.state.store(1);
        ctx->rx_used = true;                       // packet mode: drains on the copy engine
        ctx->host_copies = true;
        *rx = i;
        return 0;
    }
    return set_err(ctx, HDRF_E_CAPACITY, "every receive buffer holds a block being received or reduced (hdrf_wait_batch)");
}

extern "C" int hdrf_append_packet(hdrf_ctx *ctx, int32_t rx, const uint8_t *data, uint64_t len)
{
    if (!ctx) return HDRF_E_INVAL;
    if (rx < 0 || rx >= hdrf_ctx::kRx || ctx->rx[rx].state.load() != 1 || (len && !data)) {
        HDRF_LOCK(ctx);
        return set_err(ctx, HDRF_E_INVAL, "bad receive buffer or packet");
    }
    hdrf_ctx::Rx &r = ctx->rx[rx];
    if (len > (uint64_t)ctx->cfg.max_block_bytes - r.len) {       // r.len <= max_block_bytes: no wrap
        HDRF_LOCK(ctx);
        return set_err(ctx, HDRF_E_INVAL, "block larger than max_block_bytes");
    }
    while (len) {
        if (r.fill == 0) r.dst = r.len;
        const uint64_t n = std::min(len, ctx->kRingChunk - r.fill);
        if (rx_nt()) copy_nt(r.h + (uint64_t)r.cur * ctx->kRingChunk + r.fill, data, n);
        else std::memcpy(r.h + (uint64_t)r.cur * ctx->kRingChunk + r.fill, data, n);
        r.fill += n;
        r.len += n;
        data += n;
        len -= n;
        if (r.fill == ctx->kRingChunk) {
            const hipError_t e = rx_flush(ctx, r);
            if (e != hipSuccess) {
                HDRF_LOCK(ctx);
                return set_err(ctx, HDRF_E_HIP, std::string("packet copy: ") + hipGetErrorString(e));
            }
        }
    }
    return 0;
}

// A receive the DataNode abandons (client lost mid-block: the reference drops bf1): the buffer's
// staging copies are waited for and the buffer is free again.  The receiver thread must have
// stopped appending to it.
extern "C" int hdrf_rx_cancel(hdrf_ctx *ctx, int32_t rx)
{
    HDRF_LOCK(ctx);
    if (!ctx || rx < 0 || rx >= hdrf_ctx::kRx || ctx->rx[rx].state.load() != 1)
        return ctx ? set_err(ctx, HDRF_E_INVAL, "bad receive buffer (not receiving)") : HDRF_E_INVAL;
    hdrf_ctx::Rx &r = ctx->rx[rx];
    for (int c = 0; c < 2; c++)
        if (r.busy[c]) {
            HIPCK(hipEventSynchronize(r.ev[c]));
            r.busy[c] = false;
        }
    r.len = r.fill = r.dst = 0;
    r.cur = 0;
    r.state.store(0);
    return 0;
}

// n received blocks (receive buffers in arrival order) as ONE batch: the DataNode hands over every
// block whose last packet has arrived since its previous submit, so the batch's kernels, index and
// store passes are shared by those blocks instead of running once per block.
extern "C" int hdrf_submit_slots(hdrf_ctx *ctx, int32_t n, const int32_t *rxs)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (n < 1 || n > ctx->max_batch || !rxs) return set_err(ctx, HDRF_E_INVAL, "bad receive-buffer list");
    uint32_t mask = 0;
    for (int i = 0; i < n; i++) {
        const int32_t rx = rxs[i];
        if (rx < 0 || rx >= hdrf_ctx::kRx || ctx->rx[rx].state.load() != 1 || (mask >> rx & 1))
            return set_err(ctx, HDRF_E_INVAL, "bad receive buffer");
        mask |= 1u << rx;
    }
    if (ctx->nsub - ctx->nwait >= (uint64_t)kSlots)     // every submit pairs with one hdrf_wait_batch
        return set_err(ctx, HDRF_E_CAPACITY, "pipeline full: hdrf_wait_batch first");
    std::vector<const uint8_t *> p(n);
    std::vector<uint64_t> len(n), readable(n), id(n);
    for (int i = 0; i < n; i++) {
        hdrf_ctx::Rx &r = ctx->rx[rxs[i]];
        HIPCK(rx_flush(ctx, r));
        // (no slack fill: the kernels never depend on the bytes past a block's end, as for caller
        // buffers, and a fill kernel on the copy stream waited for CU slots and stalled the copies)
        if (r.st) {                                    // the batch's copies complete on stream C's clock
            HIPCK(hipEventRecord(r.done, r.st));
            HIPCK(hipStreamWaitEvent(ctx->stC, r.done, 0));
        }
        p[i] = r.d;
        len[i] = r.len;
        readable[i] = (uint64_t)ctx->cfg.max_block_bytes + kSlack + 256;
        id[i] = r.id;
    }
    Slot &S = ctx->sl[ctx->nsub % kSlots];
    HIPCK(hipEventRecord(S.copy_done, ctx->stC));
    if (int rc = submit(ctx, n, p.data(), len.data(), readable.data(), id.data(), true)) return rc;
    S.rx_release = mask;
    for (int i = 0; i < n; i++) ctx->rx[rxs[i]].state = 2;
    return 0;
}

extern "C" int hdrf_submit_slot(hdrf_ctx *ctx, int32_t rx)
{
    return hdrf_submit_slots(ctx, 1, &rx);
}

extern "C" int hdrf_submit_batch(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                                 const uint64_t *readable, const uint64_t *block_ids)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G > 1) return set_err(ctx, HDRF_E_INVAL, "node-global context: use the hdrf_gx_* phases");
    if (ctx->nsub - ctx->nwait >= (uint64_t)kSlots)     // every submit pairs with one hdrf_wait_batch
        return set_err(ctx, HDRF_E_CAPACITY, "pipeline full: hdrf_wait_batch first");
    return submit(ctx, nblocks, dev_data, len, readable, block_ids);
}

// Host-resident batch: the blocks are copied into the slot's device staging buffer on stream C
// (hipMemcpyAsync; overlapped with the kernels of the batches in flight when the host memory is
// pinned), then reduced exactly like hdrf_submit_batch.
extern "C" int hdrf_submit_host(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *host_data, const uint64_t *len,
                                const uint64_t *block_ids)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G > 1) return set_err(ctx, HDRF_E_INVAL, "node-global context: use the hdrf_gx_* phases");
    if (nblocks < 1 || nblocks > ctx->max_batch || !host_data || !len) return set_err(ctx, HDRF_E_INVAL, "bad batch arguments");
    for (int b = 0; b < nblocks; b++) {
        if ((int64_t)len[b] > ctx->cfg.max_block_bytes) return set_err(ctx, HDRF_E_INVAL, "block larger than max_block_bytes");
        if (len[b] && !host_data[b]) return set_err(ctx, HDRF_E_INVAL, "null block data");
    }
    if (ctx->nsub - ctx->nwait >= (uint64_t)kSlots)     // every submit pairs with one hdrf_wait_batch
        return set_err(ctx, HDRF_E_CAPACITY, "pipeline full: hdrf_wait_batch first");
    Slot &S = ctx->sl[ctx->nsub % kSlots];
    ctx->host_copies = true;
    const uint64_t stride = ((uint64_t)ctx->cfg.max_block_bytes + kSlack + 255) & ~(uint64_t)255;
    if (!S.d_hstage) {                                 // first host batch of this slot
        HIPCK(hipMalloc((void **)&S.d_hstage, stride * ctx->max_batch));
        S.hstage_stride = stride;
    }
    std::vector<const uint8_t *> ptrs(nblocks);
    std::vector<uint64_t> rd(nblocks);
    for (int b = 0; b < nblocks; b++) {
        uint8_t *d = S.d_hstage + (uint64_t)b * stride;
        // Only the copies go on stream C.  The 64 readable bytes past the block end are not filled:
        // the kernels never depend on them (device batches hand over arbitrary bytes there, e.g. the
        // next block), and a fill kernel between the copies waited for CU slots behind the drain and
        // the reduction, stalling the copy engine 8-10 ms per 16-block batch (config 5 trace, r04).
        if (len[b]) HIPCK(hipMemcpyAsync(d, host_data[b], len[b], hipMemcpyHostToDevice, ctx->stC));
        ptrs[b] = d;
        rd[b] = stride * (uint64_t)(ctx->max_batch - b);
    }
    HIPCK(hipEventRecord(S.copy_done, ctx->stC));
    return submit(ctx, nblocks, ptrs.data(), len, rd.data(), block_ids, true);
}

static int grow(hdrf_ctx *ctx, uint8_t **p, uint64_t *cap, uint64_t need);

// Stream mode (compressor 4 / 0, DN/BlockReceiver.java:826-873,887-894,1238-1256): the block as
// codec.createOutputStream(file).write(packet) per received packet, then close().  The
// BlockCompressorStream decisions (hadoop-common 3.1.0) depend only on the write sizes, so the
// host plans the pieces (groups of buffered packets, or <= MAX_INPUT slices of one large write)
// and the GPU compresses all pieces of the block at once (one wave per piece), then frames them.
// BlockCompressorStream MAX_INPUT = bufferSize - compressionOverhead (256 KiB buffers): Lz4Codec
// overhead bufferSize/255 + 16, SnappyCodec bufferSize/6 + 32 (hadoop-common 3.1.0)
static int64_t stream_max_input(int codec)
{
    if (codec == 3) return 262144 - ((262144 >> 4) + 64 + 3);    // hadoop-lzo LzopOutputStream (LZO1X)
    return codec == 0 ? 262144 - (262144 / 6 + 32) : 262144 - (262144 / 255 + 16);
}

// hadoop-lzo LzopOutputStream.writeLzopHeader: magic, {version 0x1010, LZO library version 0x20a0
// (LZO 2.10), compat 0x0940, LZO1X_1 = method 1 / level 5, flags 0, mode 0x81a4, mtime, gmtdiff 0,
// no file name} and its Adler-32 (the reference's mtime is the wall clock: hdrf_set_lzop_mtime)
static size_t lzop_header(uint32_t mtime, uint8_t *dst)
{
    static const uint8_t magic[9] = {0x89, 'L', 'Z', 'O', 0x00, 0x0d, 0x0a, 0x1a, 0x0a};
    uint8_t h[25] = {0x10, 0x10, 0x20, 0xa0, 0x09, 0x40, 1, 5, 0, 0, 0, 0, 0, 0, 0x81, 0xa4,
                     (uint8_t)(mtime >> 24), (uint8_t)(mtime >> 16), (uint8_t)(mtime >> 8), (uint8_t)mtime, 0, 0, 0, 0, 0};
    uint32_t a = 1, b = 0;
    for (uint8_t c : h) { a = (a + c) % 65521u; b = (b + a) % 65521u; }
    const uint32_t ck = (b << 16) | a;
    std::memcpy(dst, magic, 9);
    std::memcpy(dst + 9, h, 25);
    dst[34] = (uint8_t)(ck >> 24); dst[35] = (uint8_t)(ck >> 16); dst[36] = (uint8_t)(ck >> 8); dst[37] = (uint8_t)ck;
    return 38;
}

// Stream-mode compressor 5 (GzipCodec, zlib level 6; DN/BlockReceiver.java:858-873,887-894): the
// file does not depend on the packet writes.  Stage 1 match pass, stage 2 lazy
// parse, stage 3 per-deflate-block trees + bits, stage 4 offsets / placement / CRC-32 trailer.
static int grow(hdrf_ctx *ctx, uint8_t **p, uint64_t *cap, uint64_t need);
static int64_t stream_gzip(hdrf_ctx *ctx, uint64_t block_id, const uint8_t *dev_data, uint64_t len, uint8_t *out,
                           int64_t cap)
{
    if (len >= (1ull << 31)) return set_err(ctx, HDRF_E_INVAL, "gzip stream: len must be < 2^31");
    if (int rc = drain(ctx)) return rc;
    hipStream_t st = ctx->st;
    const int64_t n = (int64_t)len, maxblk = n / 16383 + 2, slot = 16384 * 6 + 2048;
    const int64_t bound = n + (n >> 3) + 1024;
    const size_t sz[] = {(size_t)(4 * n + 64), (size_t)(4 * n + 64), (size_t)(4 * n + 64), (size_t)(4 * n + 68),
                         (size_t)(40 * maxblk + 64), 64, gzip_tab_bytes(), gzip_block_state_bytes() * (size_t)maxblk,
                         (size_t)(slot * maxblk), (size_t)(24 * maxblk + 64), (size_t)(8 * maxblk + 72),
                         (size_t)(4 * ((n >> 16) + 2)), (size_t)(bound + 64), gzip_parse_scratch(n)};
    constexpr int kBufs = 14;
    uint64_t at[kBufs + 1] = {0};                      // one grown scratch (ctx->d_rd), 256-B aligned parts
    for (int i = 0; i < kBufs; i++) at[i + 1] = at[i] + ((sz[i] + 255) & ~(size_t)255);
    if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, at[kBufs])) return rc;
    uint8_t *B[kBufs];
    for (int i = 0; i < kBufs; i++) B[i] = ctx->d_rd + at[i];
    std::vector<uint8_t> tab(gzip_tab_bytes());
    gzip_host_tab(tab.data());
    int64_t cnt[2] = {0, 0}, flen = 0;
    hipError_t e = hipMemcpyAsync(B[6], tab.data(), tab.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemsetAsync(B[12], 0, sz[12], st);
    if (e == hipSuccess) e = launch_gzip_match(dev_data, n, (uint32_t *)B[0], (uint32_t *)B[1], (uint32_t *)B[2], st);
    if (e == hipSuccess)
        e = launch_gzip_parse(dev_data, n, (const uint32_t *)B[1], (const uint32_t *)B[2], (uint32_t *)B[3],
                              (int64_t *)B[4], (int64_t *)B[5], B[13], st);
    if (e == hipSuccess) e = hipMemcpyAsync(cnt, B[5], 16, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess && (cnt[1] < 1 || cnt[1] > maxblk)) { return set_err(ctx, HDRF_E_DEVICE, "gzip parse block count"); }
    if (e == hipSuccess)
        e = launch_gzip_encode(dev_data, n, B[6], (const uint32_t *)B[3], (const int64_t *)B[4], (int)cnt[1], B[7], B[8],
                               slot, (int64_t *)B[9], (int64_t *)B[10], (uint32_t *)B[11], B[12], (int64_t *)B[5], st);
    if (e == hipSuccess) e = hipMemcpyAsync(&flen, B[5], 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) { return set_err(ctx, HDRF_E_HIP, std::string("gzip stream: ") + hipGetErrorString(e)); }
    if (flen > bound) { return set_err(ctx, HDRF_E_DEVICE, "gzip stream exceeded its bound"); }
    if (!out || cap < flen) { return set_err(ctx, HDRF_E_CAPACITY, "stream file needs " + std::to_string(flen) + " bytes"); }
    e = hipMemcpy(out, B[12], (size_t)flen, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return set_err(ctx, HDRF_E_HIP, "gzip D2H");
    ctx->lengths[(uint32_t)block_id] = (int64_t)len;   // SET id -> BE32(len) (:1238-1256)
    return flen;
}

extern "C" int64_t hdrf_stream_block(hdrf_ctx *ctx, int32_t codec, uint64_t block_id, const uint8_t *dev_data,
                                     uint64_t len, uint64_t readable, const uint64_t *writes, int32_t nwrites,
                                     uint8_t *out, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (codec != 4 && codec != 0 && codec != 5 && codec != 3)
        return set_err(ctx, HDRF_E_UNSUPPORTED, "stream codec: 0 (SnappyCodec), 3 (LzopCodec), 4 (Lz4Codec) and 5 (GzipCodec)");
    if (nwrites < 0 || (nwrites && !writes) || (len && !dev_data) || readable < len + kSlack)
        return set_err(ctx, HDRF_E_INVAL, "bad stream arguments (readable must be >= len + 64)");
    if (codec == 5) {
        uint64_t sum = 0;
        for (int w = 0; w < nwrites; w++) sum += writes[w];
        if (sum != len) return set_err(ctx, HDRF_E_INVAL, "write sizes do not add up to the block length");
        return stream_gzip(ctx, block_id, dev_data, len, out, cap);
    }
    const int64_t kMaxIn = stream_max_input(codec);     // BlockCompressorStream MAX_INPUT_SIZE
    std::vector<LzPiece> pieces;
    std::vector<LzOut> outs;
    uint64_t off = 0, gs = 0, lim = 0;
    auto piece = [&](uint64_t src, uint64_t n, uint32_t hval, uint32_t hlen) {
        pieces.push_back(LzPiece{src, (uint32_t)n, 0});
        outs.push_back(LzOut{0, hval, hlen});
    };
    const bool lzop = codec == 3;
    for (int w = 0; w < nwrites; w++) {
        const uint64_t n = writes[w];
        if (lzop && n == 0) continue;
        if (lim > 0 && n + lim > (uint64_t)kMaxIn) { piece(gs, lim, (uint32_t)lim, 4); lim = 0; }   // finish()
        if (n > (uint64_t)kMaxIn) {                                                               // segmented write
            for (uint64_t o = 0; o < n; o += kMaxIn) {
                const uint64_t sl = std::min<uint64_t>(kMaxIn, n - o);
                // Lz4Codec/SnappyCodec: one BE32 raw length for the whole write; LZOP: every slice
                // is its own block [BE32 raw][BE32 stored]
                if (lzop) piece(off + o, sl, (uint32_t)sl, 4u);
                else piece(off + o, sl, (uint32_t)n, o == 0 ? 4u : 0u);
            }
            off += n;
            continue;
        }
        if (lim == 0) gs = off;
        lim += n;
        off += n;
    }
    if (off != len) return set_err(ctx, HDRF_E_INVAL, "write sizes do not add up to the block length");
    const bool trailer = lzop || lim == 0;             // close(): BE32 0 when nothing is buffered (LZOP: always)
    if (lim > 0) piece(gs, lim, (uint32_t)lim, 4);
    const int n = (int)pieces.size();
    const uint64_t stride = lzop ? lzo_piece_stride() : lz4_piece_stride();
    const uint64_t a_pieces = 0, a_outs = ((uint64_t)n * sizeof(LzPiece) + 255) & ~255ull;
    const uint64_t a_clen = a_outs + (((uint64_t)n * sizeof(LzOut) + 255) & ~255ull);
    const uint64_t a_stage = a_clen + (((uint64_t)n * 4 + 255) & ~255ull);
    const uint64_t a_file = a_stage + (((uint64_t)n * stride + 255) & ~255ull);   // keeps later arrays aligned
    // snappy: every group split into independent 64 KiB fragments (pieces[i].pad = first one)
    std::vector<LzPiece> frags;
    if (codec == 0)
        for (int i = 0; i < n; i++) {
            pieces[i].pad = (uint32_t)frags.size();
            for (uint64_t o = 0; o < pieces[i].len; o += 65536)
                frags.push_back(LzPiece{pieces[i].src + o, (uint32_t)std::min<uint64_t>(65536, pieces[i].len - o), 0});
        }
    const int nf = (int)frags.size();
    const uint64_t a_frags = a_file + (((uint64_t)n * (stride + 8) + 16 + 255) & ~255ull);
    const uint64_t a_fclen = a_frags + (((uint64_t)nf * sizeof(LzPiece) + 255) & ~255ull);
    const uint64_t a_fscr = a_fclen + (((uint64_t)nf * 4 + 255) & ~255ull);
    const uint64_t need = a_fscr + (uint64_t)nf * snappy_frag_stride() + 16;
    if (int rc = drain(ctx)) return rc;
    if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, need)) return rc;
    uint8_t *R = ctx->d_rd;
    hipStream_t st = ctx->st;
    std::vector<uint32_t> clen(n);
    if (n) {
        HIPCK(hipMemcpyAsync(R + a_pieces, pieces.data(), n * sizeof(LzPiece), hipMemcpyHostToDevice, st));
        if (codec == 4) {
            HIPCK(launch_lz4_stream((const LzPiece *)(R + a_pieces), n, dev_data, R + a_stage, (uint32_t *)(R + a_clen), st));
        } else if (codec == 3) {
            HIPCK(launch_lzo_stream((const LzPiece *)(R + a_pieces), n, dev_data, R + a_stage, (uint32_t *)(R + a_clen), st));
        } else {
            if (nf) HIPCK(hipMemcpyAsync(R + a_frags, frags.data(), nf * sizeof(LzPiece), hipMemcpyHostToDevice, st));
            HIPCK(launch_snappy_stream((const LzPiece *)(R + a_pieces), n, (const LzPiece *)(R + a_frags), nf, dev_data,
                                       R + a_fscr, (uint32_t *)(R + a_fclen), R + a_stage, stride,
                                       (uint32_t *)(R + a_clen), st));
        }
        HIPCK(hipMemcpyAsync(clen.data(), R + a_clen, n * 4, hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
    }
    uint8_t hdr[64];
    const uint64_t hlen = lzop ? lzop_header(ctx->lzop_mtime, hdr) : 0;
    uint64_t pos = hlen;
    for (int i = 0; i < n; i++) {
        outs[i].dst = pos;
        pos += outs[i].hlen + 4 + clen[i];
    }
    const int64_t total = (int64_t)pos + (trailer ? 4 : 0);
    if (!out || cap < total) return set_err(ctx, HDRF_E_CAPACITY, "stream file needs " + std::to_string(total) + " bytes");
    if (hlen) std::memcpy(out, hdr, hlen);
    if (n) {
        HIPCK(hipMemcpyAsync(R + a_outs, outs.data(), n * sizeof(LzOut), hipMemcpyHostToDevice, st));
        HIPCK(launch_lz4_emit((const LzOut *)(R + a_outs), n, R + a_stage, (const uint32_t *)(R + a_clen), R + a_file, st));
        HIPCK(hipMemcpyAsync(out + hlen, R + a_file + hlen, pos - hlen, hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
    }
    if (trailer) std::memset(out + pos, 0, 4);
    ctx->lengths[(uint32_t)block_id] = (int64_t)len;   // SET id -> BE32(len) (:1238-1256)
    return total;
}

// The same for a host-resident block (the DataNode's received bytes): staged H2D, then streamed
extern "C" int64_t hdrf_stream_block_host(hdrf_ctx *ctx, int32_t codec, uint64_t block_id, const uint8_t *data,
                                          uint64_t len, const uint64_t *writes, int32_t nwrites, uint8_t *out,
                                          int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx || (len && !data)) return HDRF_E_INVAL;
    if (codec != 4 && codec != 0 && codec != 5 && codec != 3)
        return set_err(ctx, HDRF_E_UNSUPPORTED, "stream codec: 0 (SnappyCodec), 3 (LzopCodec), 4 (Lz4Codec) and 5 (GzipCodec)");
    if (int rc = drain(ctx)) return rc;
    if (int rc = grow(ctx, &ctx->d_stage, &ctx->stage_cap, len + kSlack)) return rc;
    if (len) HIPCK(hipMemcpy(ctx->d_stage, data, len, hipMemcpyHostToDevice));
    return hdrf_stream_block(ctx, codec, block_id, ctx->d_stage, len, len + kSlack, writes, nwrites, out, cap);
}

// Hadoop codec file (BlockCompressorStream framing: [BE32 raw] ([BE32 clen] block)* groups)
// -> the compressed blocks it holds.  A group's raw length is sliced at the codec's MAX_INPUT
// (Lz4Codec 261,100, SnappyCodec 218,422), exactly as the stream wrote it; false if malformed.
static bool plan_lz4_frame(const uint8_t *f, int64_t n, std::vector<LzDec> &items, uint64_t *raw_total,
                           int codec = 4)
{
    const uint64_t kMaxIn = (uint64_t)stream_max_input(codec);
    auto be32 = [&](int64_t i) { return ((uint64_t)f[i] << 24) | ((uint64_t)f[i + 1] << 16) | ((uint64_t)f[i + 2] << 8) | f[i + 3]; };
    int64_t i = 0;
    uint64_t o = 0;
    items.clear();
    while (i + 4 <= n) {
        const uint64_t total = be32(i);
        i += 4;
        uint64_t got = 0;
        while (got < total) {
            if (i + 4 > n) return false;
            const uint64_t c = be32(i);
            i += 4;
            if (i + (int64_t)c > n) return false;
            const uint64_t raw = std::min(kMaxIn, total - got);
            items.push_back(LzDec{(uint64_t)i, o + got, (uint32_t)c, (uint32_t)raw});
            i += (int64_t)c;
            got += raw;
        }
        o += total;
    }
    *raw_total = o;
    return i == n;
}

// decode a host-resident Lz4Codec file into device memory (dev_out, cap bytes); returns raw length
static int64_t decode_file(hdrf_ctx *ctx, const uint8_t *file, int64_t flen, uint8_t *dev_out, int64_t cap,
                           int codec = 4)
{
    std::vector<LzDec> items;
    uint64_t raw = 0;
    if (flen < 0 || (flen && !file) || !plan_lz4_frame(file, flen, items, &raw, codec))
        return set_err(ctx, HDRF_E_INVAL, codec == 4 ? "malformed Lz4Codec frame" : "malformed SnappyCodec frame");
    if ((int64_t)raw > cap || (raw && !dev_out)) return set_err(ctx, HDRF_E_CAPACITY, "output capacity");
    if (items.empty()) return (int64_t)raw;
    const int n = (int)items.size();
    const uint64_t o_items = 0, o_err = ((uint64_t)n * sizeof(LzDec) + 255) & ~255ull, o_file = o_err + 256;
    if (int rc = drain(ctx)) return rc;
    if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, o_file + (uint64_t)flen + 64)) return rc;
    uint8_t *R = ctx->d_rd;
    hipStream_t st = ctx->st;
    HIPCK(hipMemcpyAsync(R + o_file, file, (size_t)flen, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(R + o_items, items.data(), (size_t)n * sizeof(LzDec), hipMemcpyHostToDevice, st));
    HIPCK(hipMemsetAsync(R + o_err, 0, 4, st));
    if (codec == 4) HIPCK(launch_lz4_decode((const LzDec *)(R + o_items), n, R + o_file, dev_out, (int *)(R + o_err), st));
    else HIPCK(launch_snappy_decode((const LzDec *)(R + o_items), n, R + o_file, dev_out, (int *)(R + o_err), st));
    int err = 0;
    HIPCK(hipMemcpyAsync(&err, R + o_err, 4, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    if (err) return set_err(ctx, HDRF_E_INVAL, codec == 4 ? "corrupt LZ4 block in the Lz4Codec file"
                                                          : "corrupt snappy block in the SnappyCodec file");
    return (int64_t)raw;
}

// ---- LzopCodec read side (DN/DataConstructor.java:140-166): LzopInputStream ----------------
// header (magic, method LZO1X, Adler-32 / CRC-32 flags, optional file name; the header checksum is
// checked), then blocks [BE32 raw][BE32 stored][checksums per the flags][bytes] up to BE32 0; one
// wave per block decodes on the GPU (lzo.hip), stored == raw means the bytes are raw
static int64_t decode_lzop(hdrf_ctx *ctx, const uint8_t *f, int64_t n, uint8_t *dev_out, int64_t cap)
{
    static const uint8_t magic[9] = {0x89, 'L', 'Z', 'O', 0x00, 0x0d, 0x0a, 0x1a, 0x0a};
    auto be32 = [&](int64_t i) { return ((uint32_t)f[i] << 24) | ((uint32_t)f[i + 1] << 16) | ((uint32_t)f[i + 2] << 8) | f[i + 3]; };
    if (n < 9 + 29 || !f || std::memcmp(f, magic, 9) != 0) return set_err(ctx, HDRF_E_INVAL, "not an lzop file");
    const uint8_t *h = f + 9;
    const uint32_t flags = be32(9 + 8);
    const int fname = h[24];
    if ((h[6] != 1 && h[6] != 2 && h[6] != 3) || (flags & 0x40)) return set_err(ctx, HDRF_E_INVAL, "unsupported lzop header");
    int64_t pos = 9 + 25 + fname;
    if (pos + 4 > n) return set_err(ctx, HDRF_E_INVAL, "truncated lzop header");
    uint32_t a = 1, b = 0;
    for (int i = 0; i < 25 + fname; i++) { a = (a + h[i]) % 65521u; b = (b + a) % 65521u; }
    if (be32(pos) != ((b << 16) | a)) return set_err(ctx, HDRF_E_INVAL, "lzop header checksum mismatch");
    pos += 4;
    const int dck = ((flags & 1) != 0) + ((flags & 0x100) != 0), cck = ((flags & 2) != 0) + ((flags & 0x200) != 0);
    std::vector<LzDec> items;
    uint64_t raw = 0;
    for (;;) {
        if (pos + 4 > n) return set_err(ctx, HDRF_E_INVAL, "truncated lzop file");
        const uint32_t ul = be32(pos);
        pos += 4;
        if (ul == 0) break;
        if (pos + 4 > n) return set_err(ctx, HDRF_E_INVAL, "truncated lzop file");
        const uint32_t cl = be32(pos);
        pos += 4 + 4 * (int64_t)dck + (cl < ul ? 4 * (int64_t)cck : 0);
        if (cl > ul || pos + cl > n) return set_err(ctx, HDRF_E_INVAL, "malformed lzop block");
        items.push_back(LzDec{(uint64_t)pos, raw, cl, ul});
        pos += cl;
        raw += ul;
    }
    if (pos != n) return set_err(ctx, HDRF_E_INVAL, "bytes after the lzop end marker");
    if ((int64_t)raw > cap || (raw && !dev_out)) return set_err(ctx, HDRF_E_CAPACITY, "output capacity");
    if (items.empty()) return 0;
    const int m = (int)items.size();
    const uint64_t o_items = 0, o_err = ((uint64_t)m * sizeof(LzDec) + 255) & ~255ull, o_file = o_err + 256;
    if (int rc = drain(ctx)) return rc;
    if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, o_file + (uint64_t)n + 64)) return rc;
    uint8_t *R = ctx->d_rd;
    hipStream_t st = ctx->st;
    HIPCK(hipMemcpyAsync(R + o_file, f, (size_t)n, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(R + o_items, items.data(), (size_t)m * sizeof(LzDec), hipMemcpyHostToDevice, st));
    HIPCK(hipMemsetAsync(R + o_err, 0, 4, st));
    HIPCK(launch_lzo_decode((const LzDec *)(R + o_items), m, R + o_file, dev_out, (int *)(R + o_err), st));
    int err = 0;
    HIPCK(hipMemcpyAsync(&err, R + o_err, 4, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    if (err) return set_err(ctx, HDRF_E_INVAL, "corrupt LZO1X block in the lzop file");
    return (int64_t)raw;
}

// ---- GzipCodec read side (DN/DataConstructor.java:194-218) -----------------------------------
// CRC-32 combination over GF(2) (zlib's crc32_combine: the CRC of A||B from crc(A), crc(B), |B|)
static uint32_t gf2_times(const uint32_t *mat, uint32_t vec)
{
    uint32_t sum = 0;
    for (int i = 0; vec; vec >>= 1, i++)
        if (vec & 1) sum ^= mat[i];
    return sum;
}
static void gf2_square(uint32_t *sq, const uint32_t *mat)
{
    for (int n = 0; n < 32; n++) sq[n] = gf2_times(mat, mat[n]);
}
// the operator "append len2 zero bytes" as a 32x32 matrix (columns)
static void crc_shift_op(uint32_t *op, int64_t len2)
{
    uint32_t odd[32], even[32];
    odd[0] = 0xEDB88320u;                     // x^1 (one zero bit)
    uint32_t row = 1;
    for (int n = 1; n < 32; n++) { odd[n] = row; row <<= 1; }
    gf2_square(even, odd);                    // 2 bits
    gf2_square(odd, even);                    // 4 bits
    for (int n = 0; n < 32; n++) op[n] = 1u << n;     // identity
    uint32_t *cur = odd, *nxt = even;         // cur: the operator for 8 * 2^k bits as k grows
    // start at one byte: square twice more (8 bits)
    gf2_square(nxt, cur);                     // 8 bits in nxt
    std::swap(cur, nxt);
    while (len2) {
        if (len2 & 1) {
            uint32_t t[32];
            for (int n = 0; n < 32; n++) t[n] = gf2_times(cur, op[n]);
            std::memcpy(op, t, sizeof t);
        }
        len2 >>= 1;
        if (!len2) break;
        gf2_square(nxt, cur);
        std::swap(cur, nxt);
    }
}
static uint32_t crc_combine_op(const uint32_t *op, uint32_t crc1, uint32_t crc2) { return gf2_times(op, crc1) ^ crc2; }

static int64_t decode_gzip(hdrf_ctx *ctx, const uint8_t *file, int64_t flen, uint8_t *dev_out, int64_t cap)
{
    if (flen < 0 || (flen && !file) || cap < 0 || (cap && !dev_out)) return set_err(ctx, HDRF_E_INVAL, "bad buffers");
    if (flen == 0) return 0;                  // an empty file decodes to nothing
    if (int rc = drain(ctx)) return rc;
    constexpr int64_t kPiece = 1 << 16;       // crc32_piece_kernel's piece
    hipStream_t st = ctx->st;
    uint32_t piece_op[32];
    crc_shift_op(piece_op, kPiece);
    CrcOp op1k;
    crc_shift_op(op1k.m, 1024);
    int64_t at = 0, out = 0;
    std::vector<uint32_t> crcs;
    while (at < flen) {
        // gzip member header (RFC 1952): ID1 ID2 CM FLG MTIME(4) XFL OS [XLEN extra] [name\0] [comment\0] [CRC16]
        if (flen - at < 18 || file[at] != 0x1f || file[at + 1] != 0x8b || file[at + 2] != 8)
            return set_err(ctx, HDRF_E_INVAL, "not a gzip member at offset " + std::to_string(at));
        const uint8_t flg = file[at + 3];
        int64_t h = at + 10;
        if (flg & 4) { if (h + 2 > flen) return set_err(ctx, HDRF_E_INVAL, "gzip header"); h += 2 + (file[h] | (file[h + 1] << 8)); }
        if (flg & 8) { while (h < flen && file[h]) h++; h++; }
        if (flg & 16) { while (h < flen && file[h]) h++; h++; }
        if (flg & 2) h += 2;
        if (h > flen) return set_err(ctx, HDRF_E_INVAL, "gzip header");
        // ---- 1. speculative chunk starts + per-chunk decode counts (inflate.hip) ----------------
        const int64_t slen = flen - h, nch = inflate_chunks(slen);
        const uint64_t o_file = 0, o_st = (o_file + (uint64_t)slen + 64 + 255) & ~255ull;
        const uint64_t o_info = o_st + (((uint64_t)nch * 8 + 255) & ~255ull);
        const uint64_t o_job = o_info + (((uint64_t)nch * 32 + 255) & ~255ull);
        const uint64_t o_misc = o_job + (((uint64_t)nch * 40 + 255) & ~255ull);
        const uint64_t o_crc = o_misc + 256, o_scr = (o_crc + 4 * ((uint64_t)(cap - out) / kPiece + 2) + 255) & ~255ull;
        if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, o_scr + 256)) return rc;
        uint8_t *R = ctx->d_rd;
        HIPCK(hipMemcpyAsync(R + o_file, file + h, (size_t)slen, hipMemcpyHostToDevice, st));
        HIPCK(launch_inflate_find(R + o_file, slen, (int64_t *)(R + o_st), (int64_t *)(R + o_info), st));
        std::vector<int64_t> starts((size_t)nch), info((size_t)nch * 4);
        HIPCK(hipMemcpyAsync(starts.data(), R + o_st, 8 * (size_t)nch, hipMemcpyDeviceToHost, st));
        HIPCK(hipMemcpyAsync(info.data(), R + o_info, 32 * (size_t)nch, hipMemcpyDeviceToHost, st));
        HIPCK(hipStreamSynchronize(st));
        // ---- 2. the chain of real block boundaries from chunk 0; output offsets ----------------
        std::vector<int64_t> jobs;
        int64_t n = 0, end_bit = -1;
        for (int64_t c = 0; c < nch;) {
            const int64_t *f = &info[(size_t)c * 4];
            if (f[2] < 0 || (f[2] <= c && !f[3])) return set_err(ctx, HDRF_E_INVAL, "corrupt deflate stream");
            jobs.insert(jobs.end(), {starts[(size_t)c], f[1], n, f[0], c});
            n += f[0];
            if (f[3]) { end_bit = f[1]; break; }
            c = f[2];
        }
        if (end_bit < 0) return set_err(ctx, HDRF_E_INVAL, "deflate stream without a final block");
        if (n > cap - out) return set_err(ctx, HDRF_E_CAPACITY, "output capacity");
        const int64_t end = h + (end_bit + 7) / 8;
        if (end + 8 > flen) return set_err(ctx, HDRF_E_INVAL, "gzip trailer missing");
        const uint32_t want_crc = (uint32_t)file[end] | ((uint32_t)file[end + 1] << 8) | ((uint32_t)file[end + 2] << 16) |
                                  ((uint32_t)file[end + 3] << 24);
        const uint32_t isize = (uint32_t)file[end + 4] | ((uint32_t)file[end + 5] << 8) | ((uint32_t)file[end + 6] << 16) |
                               ((uint32_t)file[end + 7] << 24);
        if (isize != (uint32_t)n) return set_err(ctx, HDRF_E_INVAL, "gzip ISIZE mismatch");
        // ---- 3. decode the chain's chunks in parallel, resolve cross-chunk window bytes --------
        if (n > 0) {
            const int nj = (int)(jobs.size() / 5);
            if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, o_scr + 4 * (uint64_t)n + 256)) return rc;
            if (ctx->d_rd != R) {                      // regrown: the file copy moves with it
                R = ctx->d_rd;
                HIPCK(hipMemcpyAsync(R + o_file, file + h, (size_t)slen, hipMemcpyHostToDevice, st));
            }
            uint32_t *scr = (uint32_t *)(R + o_scr);
            int *d_err = (int *)(R + o_misc);
            unsigned int *d_left = (unsigned int *)(R + o_misc + 8);
            HIPCK(hipMemcpyAsync(R + o_job, jobs.data(), 8 * jobs.size(), hipMemcpyHostToDevice, st));
            HIPCK(hipMemsetAsync(R + o_misc, 0, 16, st));
            HIPCK(launch_inflate_write(R + o_file, slen, (const int64_t *)(R + o_job), nj, scr, cap - out, d_err, st));
            int herr = 0;
            HIPCK(hipMemcpyAsync(&herr, d_err, 4, hipMemcpyDeviceToHost, st));
            HIPCK(hipStreamSynchronize(st));
            if (herr) return set_err(ctx, HDRF_E_INVAL, "corrupt deflate stream (chunk decode)");
            for (int pass = 0; nj > 1; pass++) {       // pointer jumping: chains halve every pass
                if (pass > 64) return set_err(ctx, HDRF_E_DEVICE, "window markers did not resolve");
                unsigned int left = 0;
                HIPCK(hipMemsetAsync(d_left, 0, 4, st));
                HIPCK(launch_inflate_resolve(scr, n, d_left, st));
                HIPCK(hipMemcpyAsync(&left, d_left, 4, hipMemcpyDeviceToHost, st));
                HIPCK(hipStreamSynchronize(st));
                if (!left) break;
            }
            HIPCK(launch_inflate_pack(scr, n, dev_out + out, st));
        }
        // CRC-32 of this member's output: 64 KiB pieces on the GPU, combined here
        const int64_t np = (n + kPiece - 1) / kPiece;
        uint32_t crc = 0;
        if (np) {
            HIPCK(launch_crc32_pieces(dev_out + out, n, op1k, (uint32_t *)(R + o_crc), st));
            crcs.resize((size_t)np);
            HIPCK(hipMemcpyAsync(crcs.data(), R + o_crc, 4 * (size_t)np, hipMemcpyDeviceToHost, st));
            HIPCK(hipStreamSynchronize(st));
            crc = crcs[0];
            for (int64_t i = 1; i < np; i++) {
                const int64_t len2 = std::min(kPiece, n - i * kPiece);
                if (len2 == kPiece) crc = crc_combine_op(piece_op, crc, crcs[(size_t)i]);
                else {
                    uint32_t op[32];
                    crc_shift_op(op, len2);
                    crc = crc_combine_op(op, crc, crcs[(size_t)i]);
                }
            }
        }
        if (crc != want_crc) return set_err(ctx, HDRF_E_INVAL, "gzip CRC-32 mismatch");
        out += n;
        at = end + 8;
    }
    return out;
}

// Read side for files: the Lz4Codec input stream DataConstructor opens for closed containers under
// compressor 2 (DN/DataConstructor.java:495-500) and for stream-mode blocks (:171-176).
extern "C" int64_t hdrf_lz4_file_decode(hdrf_ctx *ctx, const uint8_t *file, int64_t flen, uint8_t *dev_out, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    return decode_file(ctx, file, flen, dev_out, cap);
}

// The same for a stream-mode block file of codec 0 (SnappyCodec) or 4 (Lz4Codec): DataConstructor's
// compression-only decoders (DN/DataConstructor.java:102-220)
extern "C" int64_t hdrf_stream_file_decode(hdrf_ctx *ctx, int32_t codec, const uint8_t *file, int64_t flen,
                                           uint8_t *dev_out, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (codec == 5) return decode_gzip(ctx, file, flen, dev_out, cap);
    if (codec == 3) return decode_lzop(ctx, file, flen, dev_out, cap);
    if (codec != 0 && codec != 4)
        return set_err(ctx, HDRF_E_UNSUPPORTED, "stream codec: 0 (SnappyCodec), 3 (LzopCodec), 4 (Lz4Codec), 5 (GzipCodec)");
    return decode_file(ctx, file, flen, dev_out, cap, codec);
}

extern "C" int hdrf_set_lzop_mtime(hdrf_ctx *ctx, uint32_t mtime)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    ctx->lzop_mtime = mtime;
    return 0;
}

// Compressor 5 stage 1 (gzip.hip): per-position longest_match answers for both chain limits.
extern "C" int hdrf_gzip_match_pass(hdrf_ctx *ctx, const uint8_t *dev_data, uint64_t len, uint32_t *dev_prev,
                                    uint32_t *dev_out128, uint32_t *dev_out32)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (len && (!dev_data || !dev_prev || !dev_out128 || !dev_out32)) return set_err(ctx, HDRF_E_INVAL, "null buffer");
    if (len >= (1ull << 31)) return set_err(ctx, HDRF_E_INVAL, "gzip match pass: len must be < 2^31");
    if (int rc = drain(ctx)) return rc;
    HIPCK(launch_gzip_match(dev_data, (int64_t)len, dev_prev, dev_out128, dev_out32, ctx->st));
    HIPCK(hipStreamSynchronize(ctx->st));
    return 0;
}

// Compressor 5 stage 2 (gzip.hip): the lazy parse over stage 1's answers.
extern "C" int hdrf_gzip_parse(hdrf_ctx *ctx, const uint8_t *dev_data, uint64_t len, const uint32_t *dev_m128,
                               const uint32_t *dev_m32, uint32_t *dev_syms, int64_t *dev_blks, int64_t *dev_cnt)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (!dev_syms || !dev_blks || !dev_cnt || (len && (!dev_data || !dev_m128 || !dev_m32)))
        return set_err(ctx, HDRF_E_INVAL, "null buffer");
    if (len >= (1ull << 31)) return set_err(ctx, HDRF_E_INVAL, "gzip parse: len must be < 2^31");
    if (int rc = drain(ctx)) return rc;
    if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, gzip_parse_scratch((int64_t)len))) return rc;
    hipError_t e = launch_gzip_parse(dev_data, (int64_t)len, dev_m128, dev_m32, dev_syms, dev_blks, dev_cnt, ctx->d_rd,
                                     ctx->st);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->st);
    if (e != hipSuccess) return set_err(ctx, HDRF_E_HIP, std::string("gzip parse: ") + hipGetErrorString(e));
    return 0;
}

// Make container `id` readable for reconstruction from its chunkDir file (raw, or a closed
// container's Lz4Codec file): a DataNode that restarted, or whose arena slot was reused.
extern "C" int hdrf_container_load(hdrf_ctx *ctx, uint32_t id, const uint8_t *file, int64_t flen, int32_t lz4)
{
    HDRF_LOCK(ctx);
    if (!ctx || flen < 0 || (flen && !file)) return HDRF_E_INVAL;
    uint64_t raw = (uint64_t)flen;
    if (lz4) {
        std::vector<LzDec> items;
        if (!plan_lz4_frame(file, flen, items, &raw)) return set_err(ctx, HDRF_E_INVAL, "malformed Lz4Codec frame");
    }
    if (raw > ctx->cfg.container_max) return set_err(ctx, HDRF_E_INVAL, "container larger than container_max");
    if (int rc = drain(ctx)) return rc;
    uint8_t *p = nullptr;
    HIPCK(hipMalloc((void **)&p, raw + 64));
    int64_t got = (int64_t)raw;
    if (lz4) got = decode_file(ctx, file, flen, p, (int64_t)raw);
    else if (raw) {
        if (hipMemcpy(p, file, raw, hipMemcpyHostToDevice) != hipSuccess) got = set_err(ctx, HDRF_E_HIP, "H2D copy");
    }
    if (got < 0) { (void)hipFree(p); return (int)got; }
    auto it = ctx->loaded.find(id);
    if (it != ctx->loaded.end()) (void)hipFree(it->second.ptr);
    ctx->loaded[id] = hdrf_ctx::Loaded{p, raw};
    return 0;
}

extern "C" int hdrf_container_unload(hdrf_ctx *ctx, uint32_t id)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (int rc = drain(ctx)) return rc;
    auto it = ctx->loaded.find(id);
    if (it == ctx->loaded.end()) return set_err(ctx, HDRF_E_NOTFOUND, "container not loaded");
    (void)hipFree(it->second.ptr);
    ctx->loaded.erase(it);
    return 0;
}

extern "C" int hdrf_host_alloc(hdrf_ctx *ctx, uint64_t bytes, void **out)
{
    HDRF_LOCK(ctx);
    if (!ctx || !out) return HDRF_E_INVAL;
    HIPCK(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return 0;
}

extern "C" int hdrf_host_free(hdrf_ctx *ctx, void *p)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (p) HIPCK(hipHostFree(p));
    return 0;
}

extern "C" int hdrf_wait_batch(hdrf_ctx *ctx)
{
    if (!ctx) return HDRF_E_INVAL;
    // Block on the oldest batch's completion events WITHOUT the context lock, so receiver threads
    // (hdrf_rx_begin, hdrf_submit_slot) and drains are not stalled behind a GPU wait; wait_one then
    // finds the events complete.  (Should the slot be waited and reused meanwhile, its events
    // belong to a newer batch: this only waits longer.)
    hipEvent_t ev[2] = {nullptr, nullptr};
    {
        HDRF_LOCK(ctx);
        if (ctx->nwait < ctx->nsub) {
            const Slot &S = ctx->sl[(int)(ctx->nwait % kSlots)];
            ev[0] = S.back_done;
            if (ctx->cfg.compressor == 2) ev[1] = S.lz_done;
        }
    }
    for (hipEvent_t e : ev)
        if (e) (void)hipEventSynchronize(e);           // errors are reported by wait_one below
    HDRF_LOCK(ctx);
    return wait_one(ctx);
}

extern "C" int hdrf_batch_nblocks(hdrf_ctx *ctx)
{
    HDRF_LOCK(ctx);
    return ctx ? ctx->last_nblocks : HDRF_E_INVAL;
}

extern "C" int hdrf_reduce_batch(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                                 const uint64_t *readable, const uint64_t *block_ids)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G > 1) return set_err(ctx, HDRF_E_INVAL, "node-global context: use the hdrf_gx_* phases");
    if (int rc = drain(ctx)) return rc;
    if (int rc = submit(ctx, nblocks, dev_data, len, readable, block_ids)) return rc;
    return wait_one(ctx);
}

// ---- node-global index phases (include/hdrf.h, gx.hip) ------------------------------------
static_assert(sizeof(AllocState) <= HDRF_ALLOC_STATE_BYTES, "allocator state exchange size");

// back phases run on the oldest batch whose front was waited, in order owner..commit
static int gx_check(hdrf_ctx *ctx, int bphase)
{
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G < 2) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_* needs cfg.n_ranks > 1");
    if (ctx->gx_nfwait <= ctx->gx_nback || ctx->gx_bphase != bphase)
        return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_* phases called out of order (back phase " +
                                              std::to_string(ctx->gx_bphase) + ")");
    return 0;
}

static int64_t max_count(const int64_t *counts, int G)
{
    int64_t m = 0;
    for (int i = 0; i < G; i++) m = std::max(m, counts[i]);
    return m;
}

extern "C" int hdrf_gx_layout_get(hdrf_ctx *ctx, hdrf_gx_layout *out)
{
    HDRF_LOCK(ctx);
    if (!ctx || !out) return HDRF_E_INVAL;
    out->cap = ctx->gx_cap;
    out->x1_words = ctx->HW + 2;
    out->x2_words = 2;
    out->x3_words = 4;
    out->depth = ctx->gx_depth;
    out->fn_bytes = (int64_t)ctx->fn_bytes;
    return 0;
}

// ---- node-global pipeline ----------------------------------------------------
// A batch's front half runs like the single-node pipeline: chunking on stream W, SHA on stream A,
// then the local aggregation and its X1 records on stream X, in slot seq % gx_depth, so the fronts
// of the next batches run while the oldest batch goes through its exchanges and back phases on
// stream B.  The back half enqueues without host round trips: the allocator scan runs on the
// device (hdrf_gx_flush_fn_dev -> all-gather of fixed-size descriptors -> hdrf_gx_alloc_scan_dev),
// placement and its read-back are one event the host waits for (the X3 counts size the X3
// exchange), the arena copy runs on stream B2 beside the next batch's owner phases, and the commit
// is not waited for (its errors are reported by the next place or hdrf_gx_sync).

static void gx_mark(hdrf_ctx *ctx, uint64_t seq, int e, hipStream_t st)
{
    if (!ctx->timing) return;
    GxTime &T = ctx->gxt[seq % kGxRing];
    if (hipEventRecord(T.ev[e], st) == hipSuccess) T.rec |= 1u << e;
}

// phase times of completed batches, in order (wait: block until they are complete)
static void gx_collect(hdrf_ctx *ctx, bool wait, uint64_t upto)
{
    if (!ctx->timing) return;
    while (ctx->gxt_done < upto && ctx->gxt_done < ctx->gx_nback) {
        const uint64_t k = ctx->gxt_done;
        GxTime &T = ctx->gxt[k % kGxRing];
        const auto has = [&](int e) { return (T.rec >> e & 1) != 0; };
        for (int e : {(int)kG13, (int)kP1})
            if (has(e)) {
                if (wait) (void)hipEventSynchronize(T.ev[e]);
                else if (hipEventQuery(T.ev[e]) != hipSuccess) return;
            }
        const auto add = [&](int stage, int a, int b) {
            if (has(a) && has(b)) ctx->stage_ms[stage] += elapsed(T.ev[a], T.ev[b]);
        };
        add(11, kW0, kW0 + 1); add(0, kW0 + 1, kW0 + 2); add(1, kW0 + 2, kW0 + 3);
        add(2, kA0, kA0 + 1);
        add(12, kX0, kX0 + 3);
        add(13, kG0, kG1); add(20, kG1, kG2); add(14, kG2, kG3); add(7, kG3, kG4);
        add(15, kG5, kG6); add(21, kG6, kG7); add(16, kG7, kG8); add(8, kG8, kG9);
        add(17, kG10, kG11); add(22, kG11, kG12); add(18, kG12, kG13);
        add(9, kP0, kP1);
        if (k > 0) {                                    // X1 + host gap: the previous commit to this owner phase
            GxTime &Pv = ctx->gxt[(k - 1) % kGxRing];
            if ((Pv.rec >> kG13 & 1) && has(kG0)) ctx->stage_ms[19] += elapsed(Pv.ev[kG13], T.ev[kG0]);
        }
        ctx->gxt_done++;
    }
}

// Front half of a node-global batch (chunking, SHA, local aggregation, X1 records), launched into
// slot nfront % gx_depth without waiting.  The slot's previous batch must have left it: its back
// phases (stream B) and its arena copy (stream B2) are waited for on the device.
extern "C" int hdrf_gx_front_launch(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                                    const uint64_t *readable, const uint64_t *block_ids, uint32_t gbase,
                                    uint32_t *x1_send)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G < 2) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_* needs cfg.n_ranks > 1");
    const uint64_t D = (uint64_t)ctx->gx_depth;
    if (ctx->gx_nfront - ctx->gx_nback >= D)
        return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_front_launch: " + std::to_string(D) +
                                              " batches in the node-global pipeline (commit the oldest first)");
    if (!x1_send) return set_err(ctx, HDRF_E_INVAL, "null exchange buffer");
    const uint64_t seq = ctx->gx_nfront;
    const int si = (int)(seq % D);
    Slot &S = ctx->sl[si];
    const hdrf_cfg &c = ctx->cfg;
    // the timing ring entry is reused: the batch kGxRing - 1 back (and everything before) is collected
    if (ctx->timing) {
        if (seq + 2 > (uint64_t)kGxRing) gx_collect(ctx, true, seq + 2 - kGxRing);
        ctx->gxt[seq % kGxRing].rec = 0;
    }
    hipStream_t W = ctx->stW, A = ctx->st, X = ctx->stX;
    if (S.gx_inuse) {                                   // the slot's previous batch is done with it
        HIPCK(hipStreamWaitEvent(W, S.back_done, 0));
        if (S.gx_split) HIPCK(hipStreamWaitEvent(W, S.placed, 0));
    }
    if (int rc = prepare_blocks(ctx, S, nblocks, dev_data, len, readable)) return rc;
    S.gx_batch = ++ctx->batch;
    HIPCK(hipMemcpyAsync(S.d_blocks, S.h_desc, sizeof(BlockDesc) * nblocks, hipMemcpyHostToDevice, W));
    GxTime &T = ctx->gxt[seq % kGxRing];
    Marker mw, ma, mx;
    mw.ev = ctx->timing ? &T.ev[kW0] : nullptr;
    HIPCK(launch_chunking(S.d_blocks, nblocks, S.max_len, S.max_nseg, S.total_waves, S.total_segs,
                          chunk_scratch(S, c.compressor), c.window, c.max_chunk, S.d_spec, S.spec_cap, S.d_meta, S.d_bst,
                          S.d_off, ctx->cap_blk, S.d_err, W, &mw));
    mw.mark(W);
    HIPCK(hipEventRecord(S.walk_done, W));
    HIPCK(hipStreamWaitEvent(A, S.walk_done, 0));
    if (S.recipe_pending) HIPCK(hipStreamWaitEvent(A, S.recipe_done, 0));
    ma.ev = ctx->timing ? &T.ev[kA0] : nullptr;
    HIPCK(launch_sha(c.hasher, S.d_blocks, nblocks, S.d_off, S.d_bst, ctx->cap_blk, S.d_dig, S.d_queue, ctx->sha_long, A,
                     &ma));
    ma.mark(A);
    HIPCK(hipEventRecord(S.idx_done, A));               // (node-global: "the batch's digests are ready")
    // local aggregation: a fresh scratch table (the next epoch of the slot's table, cleared every 255
    // uses), every entry "created" in batch 1
    HIPCK(hipStreamWaitEvent(X, S.idx_done, 0));
    if (++ctx->scratch_epoch[si] > 255) {
        HIPCK(hipMemsetAsync(ctx->d_scratch[si], 0, sizeof(IndexEntry) << ctx->scratch_log2, X));
        ctx->scratch_epoch[si] = 1;
    }
    const unsigned long long skey = ((unsigned long long)ctx->scratch_epoch[si] << 56) | tag_bits(ctx);
    mx.ev = ctx->timing ? &T.ev[kX0] : nullptr;
    HIPCK(launch_index(c.hasher, S.d_bst, nblocks, ctx->cap_blk, S.d_off, S.d_dig, ctx->d_scratch[si],
                       ctx->scratch_log2, 1u, 1u, skey, S.d_slot, S.d_coll, S.d_ncoll, ctx->coll_cap,
                       S.d_flags, S.d_tilesum, ctx->ntiles, S.d_err, X, &mx));
    HIPCK(launch_gx_emit(c.hasher, S.d_bst, nblocks, ctx->cap_blk, ctx->ntiles, S.d_dig, ctx->d_scratch[si],
                         S.d_slot, S.d_flags, gbase, ctx->G, x1_send, ctx->gx_cap, ctx->d_gxe[si], S.d_err, X));
    mx.mark(X);
    HIPCK(hipMemcpyAsync(S.h_gx->front_cnt, ctx->d_gxe[si], sizeof(unsigned long long) * ctx->G, hipMemcpyDeviceToHost, X));
    HIPCK(hipMemcpyAsync(&S.h_gx->front_err, S.d_err, sizeof(int), hipMemcpyDeviceToHost, X));
    HIPCK(hipEventRecord(S.front_done, X));
    if (ctx->timing) T.rec |= 0xFu << kW0 | 0x7u << kA0 | 0xFu << kX0;
    S.nblocks = nblocks;
    S.lens.assign(len, len + nblocks);
    S.ids.assign(nblocks, 0);
    if (block_ids) S.ids.assign(block_ids, block_ids + nblocks);
    S.gx_inuse = true;
    S.gx_split = false;
    S.gen_reset = ctx->gen_pending;                    // the first batch of a fresh generation (hdrf_reset_async)
    ctx->gen_pending = false;
    ctx->gx_nfront++;
    return 0;
}

// Wait for the oldest launched front; its per-peer X1 record counts -> send_counts[G].
extern "C" int hdrf_gx_front_wait(hdrf_ctx *ctx, int64_t *send_counts)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->gx_nfront <= ctx->gx_nfwait) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_front_wait: no front pending");
    if (!send_counts) return set_err(ctx, HDRF_E_INVAL, "null counts");
    const int si = (int)(ctx->gx_nfwait % (uint64_t)ctx->gx_depth);
    Slot &S = ctx->sl[si];
    HIPCK(hipEventSynchronize(S.front_done));
    ctx->gx_nfwait++;
    const int herr = S.h_gx->front_err;
    if (herr) {
        HIPCK(hipMemsetAsync(S.d_err, 0, sizeof(int), ctx->stX));
        HIPCK(hipStreamSynchronize(ctx->stX));
        return device_error(ctx, herr);
    }
    S.gx_c1.assign(ctx->G, 0);
    for (int d = 0; d < ctx->G; d++) send_counts[d] = S.gx_c1[(size_t)d] = (int64_t)S.h_gx->front_cnt[d];
    return 0;
}

extern "C" int hdrf_gx_front(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                             const uint64_t *readable, const uint64_t *block_ids, uint32_t gbase, uint32_t *x1_send,
                             int64_t *send_counts)
{
    HDRF_LOCK(ctx);
    if (!send_counts) return ctx ? set_err(ctx, HDRF_E_INVAL, "null counts") : HDRF_E_INVAL;
    if (ctx && ctx->gx_nfront != ctx->gx_nfwait)
        return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_front: launched fronts are pending (hdrf_gx_front_wait)");
    if (int rc = hdrf_gx_front_launch(ctx, nblocks, dev_data, len, readable, block_ids, gbase, x1_send)) return rc;
    return hdrf_gx_front_wait(ctx, send_counts);
}

static Slot &gx_back_slot(hdrf_ctx *ctx) { return ctx->sl[ctx->gx_nback % (uint64_t)ctx->gx_depth]; }
static int gx_back_si(hdrf_ctx *ctx) { return (int)(ctx->gx_nback % (uint64_t)ctx->gx_depth); }

extern "C" int hdrf_gx_owner(hdrf_ctx *ctx, const uint32_t *x1_recv, const int64_t *recv_counts, uint32_t *x2_send)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 0)) return rc;
    Slot &S = gx_back_slot(ctx);
    if (!x1_recv || !recv_counts || !x2_send) return set_err(ctx, HDRF_E_INVAL, "null exchange buffer");
    for (int s = 0; s < ctx->G; s++)
        if (recv_counts[s] < 0 || recv_counts[s] > ctx->gx_cap) return set_err(ctx, HDRF_E_INVAL, "bad receive count");
    hipStream_t st = ctx->stB;
    const uint64_t seq = ctx->gx_nback;
    if (S.gen_reset) {
        // a fresh generation (hdrf_reset_async): the next epoch of the partition's tag words (the table
        // cleared when it wraps), batches from this one on are this generation's, and the node's
        // allocator re-seeded — on stream B after every older batch's owner..commit phases, and after
        // the last arena copy on B2 (the new generation reuses the slot rings from their start)
        hipEvent_t b2;                                 // everything on B2 so far: older batches' copies
        HIPCK(hipEventCreateWithFlags(&b2, hipEventDisableTiming));
        HIPCK(hipEventRecord(b2, ctx->stB2));
        HIPCK(hipStreamWaitEvent(st, b2, 0));
        HIPCK(hipEventDestroy(b2));
        const bool clear = ctx->epoch >= 255;
        ctx->epoch = clear ? 1 : ctx->epoch + 1;
        ctx->bfirst = S.gx_batch;
        HIPCK(launch_index_clear(ctx->d_tab, clear ? ctx->cfg.index_log2 : -1, ctx->d_alloc, initial_alloc(ctx), st, 0u));
        ctx->h_alloc = initial_alloc(ctx);            // (hdrf_gx_alloc_scan, host form, starts from it)
    }
    gx_mark(ctx, seq, kG0, st);
    std::memcpy(S.h_gx->up_r1, recv_counts, sizeof(int64_t) * ctx->G);
    HIPCK(hipMemcpyAsync(ctx->d_gx_rcounts, S.h_gx->up_r1, sizeof(int64_t) * ctx->G, hipMemcpyHostToDevice, st));
    HIPCK(hipMemsetAsync(ctx->d_gx_x3exp, 0, sizeof(unsigned long long) * ctx->G, st));
    HIPCK(launch_gx_owner(ctx->cfg.hasher, x1_recv, ctx->d_gx_rcounts, max_count(recv_counts, ctx->G), ctx->gx_cap,
                          ctx->G, ctx->d_tab, ctx->cfg.index_log2, S.gx_batch, ctx->bfirst, tag_mask(ctx), ctx->d_oslot,
                          ctx->d_oflags, S.d_coll, S.d_ncoll, ctx->coll_cap, x2_send, ctx->d_gx_x3exp, S.d_err, st));
    gx_mark(ctx, seq, kG1, st);
    // no host round trip: a device error (S.d_err) is read back with the batch by hdrf_gx_place, and
    // the X2 exchange may be enqueued on stream B right behind this kernel (hdrf_gx_stream)
    ctx->gx_bphase = 1;
    return 0;
}

extern "C" int hdrf_gx_stream(hdrf_ctx *ctx, void **stream)
{
    HDRF_LOCK(ctx);
    if (!ctx || !stream) return HDRF_E_INVAL;
    *stream = (void *)ctx->stB;
    return 0;
}

extern "C" int hdrf_gx_decide(hdrf_ctx *ctx, const uint32_t *x2_recv)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 1)) return rc;
    const int si = gx_back_si(ctx);
    Slot &S = ctx->sl[si];
    if (!x2_recv) return set_err(ctx, HDRF_E_INVAL, "null exchange buffer");
    hipStream_t st = ctx->stB;
    const uint64_t seq = ctx->gx_nback;
    const int nb = S.nblocks;
    gx_mark(ctx, seq, kG2, st);
    HIPCK(launch_gx_decide(S.d_bst, nb, ctx->cap_blk, ctx->ntiles, S.d_off, ctx->d_scratch[si], S.d_slot, x2_recv,
                           S.d_flags, S.d_tilesum, st));
    // the X3 records the owners' answers call for (checked against place_kernel's own counts)
    HIPCK(launch_gx_x3want(x2_recv, ctx->d_gxe[si], max_count(S.gx_c1.data(), ctx->G), ctx->gx_cap, ctx->G,
                           ctx->d_x3want, st));
    gx_mark(ctx, seq, kG3, st);
    const StoreParams P = store_params(ctx, nb);
    HIPCK(launch_store_scan(P, S.d_bst, S.d_off, S.d_flags, S.d_tilesum, S.d_tilepre, S.d_store,
                            S.d_pre, st));
    gx_mark(ctx, seq, kG4, st);
    ctx->gx_x2 = x2_recv;
    ctx->gx_bphase = 2;
    return 0;
}

extern "C" int hdrf_gx_flush(hdrf_ctx *ctx, const uint8_t *alloc_in, uint8_t *alloc_out)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 2)) return rc;
    Slot &S = gx_back_slot(ctx);
    hipStream_t st = ctx->stB;
    if (alloc_in) {
        ctx->gx_dscan = 0;                             // a host-given allocator replaces the device scan's
        std::memcpy(&ctx->gx_ain, alloc_in, sizeof(AllocState));
        S.h_gx->st[0] = ctx->gx_ain;
        HIPCK(hipMemcpyAsync(ctx->d_alloc, &S.h_gx->st[0], sizeof(AllocState), hipMemcpyHostToDevice, st));
    } else if (!ctx->gx_dscan) {
        HIPCK(hipMemcpyAsync(&S.h_gx->st[0], ctx->d_alloc, sizeof(AllocState), hipMemcpyDeviceToHost, st));
    }
    HIPCK(hipMemsetAsync(S.d_nclosed, 0, sizeof(uint32_t), st));
    const StoreParams P = store_params(ctx, S.nblocks);
    HIPCK(launch_store_flush(P, S.d_bst, S.d_store, S.d_pre, ctx->d_alloc, S.d_rstate, S.d_ev,
                             S.d_closed, S.d_nclosed, S.d_err, st));
    gx_mark(ctx, ctx->gx_nback, kG9, st);
    if (!alloc_out && (ctx->gx_scanned || ctx->gx_dscan)) {   // the scan knows the result: no host round trip
        if (ctx->gx_scanned) ctx->gx_aout = ctx->gx_expect;
        ctx->gx_bphase = 3;
        return 0;
    }
    AllocState a{};
    HIPCK(hipMemcpyAsync(&S.h_gx->st[3], ctx->d_alloc, sizeof a, hipMemcpyDeviceToHost, st));
    if (ctx->gx_dscan) HIPCK(hipMemcpyAsync(S.h_gx->st, ctx->d_gxst, 2 * sizeof a, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    a = S.h_gx->st[3];
    if (!alloc_in) ctx->gx_ain = S.h_gx->st[0];
    ctx->gx_aout = a;
    if (ctx->gx_scanned && std::memcmp(&a, &ctx->gx_expect, sizeof a) != 0)
        return set_err(ctx, HDRF_E_DEVICE, "allocator scan disagrees with the flush walk");
    if (ctx->gx_dscan && std::memcmp(&a, &S.h_gx->st[1], sizeof a) != 0)
        return set_err(ctx, HDRF_E_DEVICE, "device allocator scan disagrees with the flush walk");
    if (alloc_out) {
        std::memset(alloc_out, 0, HDRF_ALLOC_STATE_BYTES);
        std::memcpy(alloc_out, &a, sizeof a);
    }
    ctx->gx_bphase = 3;
    return 0;
}

// ---- allocator scan: every rank's flush walk as a function of the incoming allocator ------
// (store.hip fn_info / fn_chain).  Host descriptor, int64 words: n_thread, then per range t
// {any, S, base_last, S_last, m, m x (v, final container start, closes after the first)}.
static int grow(hdrf_ctx *ctx, uint8_t **p, uint64_t *cap, uint64_t need);

// fn_info / fn_chain into the context's scratch (the candidate rows per range); returns the scratch
static int gx_flush_rows(hdrf_ctx *ctx, Slot &S, int *err, uint8_t **F_out)
{
    hipStream_t st = ctx->stB;
    const StoreParams P = store_params(ctx, S.nblocks);
    const int64_t kcap = (int64_t)ctx->max_batch * ctx->cap_blk + 1;
    const uint64_t o_fr = 64 * 4 * sizeof(FnBlock), o_k = o_fr + 256, o_out = o_k + 256;
    if (int rc = grow(ctx, &ctx->d_fn, &ctx->fn_cap, o_out + (uint64_t)P.n_thread * kcap * 24)) return rc;
    uint8_t *F = ctx->d_fn;
    HIPCK(hipMemsetAsync(F + o_k, 0, 64, st));
    HIPCK(launch_flush_fn(P, S.d_bst, S.d_store, S.d_pre, (FnBlock *)F, (FnRange *)(F + o_fr), (uint64_t *)(F + o_out),
                          kcap, (unsigned long long *)(F + o_k), err, st));
    *F_out = F;
    return 0;
}

extern "C" int64_t hdrf_gx_flush_fn(hdrf_ctx *ctx, int64_t *desc, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 2)) return rc;
    Slot &S = gx_back_slot(ctx);
    hipStream_t st = ctx->stB;
    const int nt = ctx->cfg.n_thread;
    const int64_t kcap = (int64_t)ctx->max_batch * ctx->cap_blk + 1;
    const uint64_t o_fr = 64 * 4 * sizeof(FnBlock), o_k = o_fr + 256, o_out = o_k + 256;
    uint8_t *F = nullptr;
    // (the function's own error word after the rows; read back with the rows' counts)
    if (int rc = grow(ctx, &ctx->d_fn, &ctx->fn_cap, o_out + (uint64_t)nt * kcap * 24 + 64)) return rc;
    int *d_err = (int *)(ctx->d_fn + o_out + (uint64_t)nt * kcap * 24);
    HIPCK(hipMemsetAsync(d_err, 0, sizeof(int), st));
    if (int rc = gx_flush_rows(ctx, S, d_err, &F)) return rc;
    FnRange fr[4];
    unsigned long long K[4];
    int herr = 0;
    HIPCK(hipMemcpyAsync(fr, F + o_fr, sizeof(FnRange) * nt, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(K, F + o_k, 8 * nt, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(&herr, d_err, 4, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    if (herr) return set_err(ctx, HDRF_E_DEVICE, "flush function: candidate table overflow or runaway chain");
    std::vector<uint64_t> rows[4];
    for (int t = 0; t < nt; t++) {
        rows[t].resize(3 * K[t]);
        if (K[t]) HIPCK(hipMemcpyAsync(rows[t].data(), F + o_out + (uint64_t)t * kcap * 24, 24 * K[t], hipMemcpyDeviceToHost, st));
    }
    HIPCK(hipStreamSynchronize(st));
    std::vector<int64_t> d{nt};
    for (int t = 0; t < nt; t++) {
        const size_t h = d.size();
        d.insert(d.end(), {(int64_t)fr[t].any, (int64_t)fr[t].S, (int64_t)fr[t].base_last, (int64_t)fr[t].S_last, 0});
        int64_t m = 0;
        for (uint64_t i = 0; i < K[t]; i++) {
            const uint64_t *r = &rows[t][3 * i];
            if (r[2] >> 63) continue;                      // repeats the previous prefix
            d.insert(d.end(), {(int64_t)r[0], (int64_t)r[1], (int64_t)r[2]});
            m++;
        }
        if (fr[t].any && (m == 0 || d[h + 5] != 0)) return set_err(ctx, HDRF_E_DEVICE, "flush function: no start candidate");
        d[h + 4] = m;
    }
    if (!desc || cap < (int64_t)d.size()) {
        if (cap >= 0) set_err(ctx, HDRF_E_CAPACITY, "flush descriptor needs " + std::to_string(d.size()) + " words");
        return -(int64_t)d.size() - 1000;           // callers size with the returned -(n + 1000)
    }
    std::copy(d.begin(), d.end(), desc);
    return (int64_t)d.size();
}

// The same function packed on the device into a fixed-size descriptor of hdrf_gx_layout.fn_bytes
// (store.hip fn_pack_kernel), enqueued on the back stream: the ranks all-gather the descriptors
// there and hdrf_gx_alloc_scan_dev composes them, with no host round trip.
extern "C" int hdrf_gx_flush_fn_dev(hdrf_ctx *ctx, void *dev_desc)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 2)) return rc;
    if (!dev_desc) return set_err(ctx, HDRF_E_INVAL, "null descriptor buffer");
    Slot &S = gx_back_slot(ctx);
    hipStream_t st = ctx->stB;
    const int nt = ctx->cfg.n_thread;
    const int64_t kcap = (int64_t)ctx->max_batch * ctx->cap_blk + 1;
    const uint64_t o_fr = 64 * 4 * sizeof(FnBlock), o_k = o_fr + 256, o_out = o_k + 256;
    gx_mark(ctx, ctx->gx_nback, kG5, st);
    uint8_t *F = nullptr;
    if (int rc = gx_flush_rows(ctx, S, S.d_err, &F)) return rc;
    HIPCK(launch_fn_pack(nt, (const FnRange *)(F + o_fr), (const uint64_t *)(F + o_out), kcap,
                         (const unsigned long long *)(F + o_k), ctx->fn_mcap, dev_desc, S.d_err, st));
    gx_mark(ctx, ctx->gx_nback, kG6, st);
    return 0;
}

// one rank's flush function applied to the allocator A (the walk of store.hip flush_kernel)
static bool gx_apply_fn(const hdrf_ctx *ctx, const int64_t *d, int64_t len, AllocState &A)
{
    if (len < 1) return false;
    const int nt = (int)d[0];
    if (nt != ctx->cfg.n_thread) return false;
    const int64_t cmax = (int64_t)ctx->cfg.container_max;
    const uint32_t per = (uint32_t)(ctx->cfg.arena_slots / 4);
    int64_t p = 1;
    for (int t = 0; t < nt; t++) {
        if (p + 5 > len) return false;
        const int64_t any = d[p], S = d[p + 1], bl = d[p + 2], Sl = d[p + 3], m = d[p + 4];
        const int64_t *v = d + p + 5;
        p += 5 + 3 * m;
        if (m < 0 || p > len) return false;
        if (!any) continue;
        const int64_t x = A.exists[t] ? (int64_t)A.cur[t] : 0;
        int64_t cs = -x, n = 0;
        if (x + S > cmax) {
            const int64_t thr = cmax - x;              // first close after the last prefix <= thr
            int64_t lo = 0, hi = m;                    // largest v <= thr (v_0 = 0 <= thr)
            while (hi - lo > 1) {
                const int64_t mid = (lo + hi) / 2;
                if (v[3 * mid] <= thr) lo = mid; else hi = mid;
            }
            cs = v[3 * lo + 1];
            n = 1 + v[3 * lo + 2];
        }
        const uint32_t base = (uint32_t)t * per;
        A.id[t] += (uint32_t)n;
        A.slot[t] = base + (uint32_t)(((int64_t)(A.slot[t] - base) + n) % per);
        A.cur[t] = (uint32_t)(S - cs);
        A.exists[t] = 1;
        A.pos[t] = (uint32_t)(Sl - std::max<int64_t>(cs - bl, 0));
    }
    return p == len;
}

// The node's allocator for this batch from every rank's flush function (rank order): the state
// this rank's flush walk starts from (the exclusive scan) and the state after the last rank.
extern "C" int hdrf_gx_alloc_scan(hdrf_ctx *ctx, const int64_t *descs, const int64_t *lens, uint8_t *alloc_in,
                                  uint8_t *alloc_final)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 2)) return rc;
    if (!descs || !lens || !alloc_in || !alloc_final) return set_err(ctx, HDRF_E_INVAL, "null scan argument");
    AllocState A = ctx->h_alloc;
    int64_t off = 0;
    for (int r = 0; r < ctx->G; r++) {
        if (r == ctx->cfg.rank) {
            std::memset(alloc_in, 0, HDRF_ALLOC_STATE_BYTES);
            std::memcpy(alloc_in, &A, sizeof A);
        }
        if (lens[r] < 1 || !gx_apply_fn(ctx, descs + off, lens[r], A))
            return set_err(ctx, HDRF_E_INVAL, "malformed flush descriptor of rank " + std::to_string(r));
        if (r == ctx->cfg.rank) ctx->gx_expect = A;
        off += lens[r];
    }
    std::memset(alloc_final, 0, HDRF_ALLOC_STATE_BYTES);
    std::memcpy(alloc_final, &A, sizeof A);
    ctx->gx_scanned = 1;
    return 0;
}

// The same composition on the device over the all-gathered descriptors (G x fn_bytes, rank order):
// the node's allocator after the previous batch (on the device already) -> this rank's incoming
// state for hdrf_gx_flush(ctx, NULL, NULL), its predicted result (checked by hdrf_gx_place) and the
// node's state after the batch (installed by hdrf_gx_place).  Enqueued on the back stream.
extern "C" int hdrf_gx_alloc_scan_dev(hdrf_ctx *ctx, const void *dev_descs)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 2)) return rc;
    if (!dev_descs) return set_err(ctx, HDRF_E_INVAL, "null descriptors");
    Slot &S = gx_back_slot(ctx);
    hipStream_t st = ctx->stB;
    gx_mark(ctx, ctx->gx_nback, kG7, st);
    HIPCK(launch_gx_scan(dev_descs, ctx->fn_bytes, ctx->G, ctx->cfg.rank, ctx->cfg.n_thread,
                         (uint32_t)(ctx->cfg.arena_slots / 4), ctx->cfg.container_max, ctx->d_alloc, ctx->d_gxst,
                         S.d_err, st));
    gx_mark(ctx, ctx->gx_nback, kG8, st);
    ctx->gx_dscan = 1;
    ctx->gx_scanned = 0;
    return 0;
}

// Placement of the back batch: on stream B the per-chunk container positions, the X3 location
// records and the read-back the host needs (hdrf_gx_place_wait); the arena copy of the new chunks
// runs on stream B2 (compressor 2 keeps it on B: its LZ4 pass reads the containers there).
extern "C" int hdrf_gx_place_launch(hdrf_ctx *ctx, const uint8_t *alloc_final, uint32_t *x3_send)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 3)) return rc;
    if (ctx->gx_place_pending) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_place_launch: a placement is pending");
    const int si = gx_back_si(ctx);
    Slot &S = ctx->sl[si];
    if (!x3_send) return set_err(ctx, HDRF_E_INVAL, "null exchange buffer");
    if (!alloc_final && !ctx->gx_dscan)
        return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_place: the node's allocator (alloc_final) is needed without the device scan");
    hipStream_t st = ctx->stB;
    const uint64_t seq = ctx->gx_nback;
    const int nb = S.nblocks;
    const StoreParams P = store_params(ctx, nb);
    const bool split = ctx->cfg.compressor != 2;
    GxPlace gx;
    gx.x2 = ctx->gx_x2; gx.x3 = x3_send; gx.cap = ctx->gx_cap; gx.counts = ctx->d_gx_counts; gx.G = ctx->G;
    gx.part = split ? 1 : 0;
    gx_mark(ctx, seq, kG10, st);
    HIPCK(launch_store_place(P, S.d_blocks, S.d_bst, S.d_off, S.d_flags, S.d_pre, S.d_rstate, S.d_ev, S.d_slot,
                             ctx->d_scratch[si], ctx->d_arena, S.d_pcid, S.d_ppos, gx, st));
    // the flush walk's result (checked against the scan), then the node's allocator after the batch
    // (the next batch and the "blockID" view start from it)
    HIPCK(hipMemcpyAsync(ctx->d_gxst + 3, ctx->d_alloc, sizeof(AllocState), hipMemcpyDeviceToDevice, st));
    if (alloc_final) {
        std::memcpy(&S.h_gx->st[2], alloc_final, sizeof(AllocState));
        HIPCK(hipMemcpyAsync(ctx->d_alloc, &S.h_gx->st[2], sizeof(AllocState), hipMemcpyHostToDevice, st));
    } else {
        HIPCK(hipMemcpyAsync(ctx->d_alloc, ctx->d_gxst + 2, sizeof(AllocState), hipMemcpyDeviceToDevice, st));
    }
    GxHost *h = S.h_gx;
    HIPCK(hipMemcpyAsync(h->c3, ctx->d_gx_counts, sizeof(unsigned long long) * ctx->G, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(h->x3e, ctx->d_gx_x3exp, sizeof(unsigned long long) * ctx->G, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(h->x3want, ctx->d_x3want, sizeof(unsigned long long) * ctx->G, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(&h->commit_err, ctx->d_gx_err, sizeof(int), hipMemcpyDeviceToHost, st));
    if (ctx->gx_dscan) HIPCK(hipMemcpyAsync(h->st, ctx->d_gxst, 2 * sizeof(AllocState), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(&h->st[3], ctx->d_gxst + 3, sizeof(AllocState), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(S.h_bst, S.d_bst, sizeof(BlockState) * nb, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(S.h_store, S.d_store, sizeof(uint64_t) * nb, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(S.h_alloc, ctx->d_alloc, sizeof(AllocState), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(S.h_err, S.d_err, sizeof(int), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(S.h_nclosed, S.d_nclosed, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(S.h_closed, S.d_closed, sizeof(ClosedRec) * ctx->closed_cap, hipMemcpyDeviceToHost, st));
    gx_mark(ctx, seq, kG11, st);
    HIPCK(hipEventRecord(S.gx_meta, st));
    if (split) {                                        // the arena copy beside the next batch's owner phases
        hipStream_t B2 = ctx->stB2;
        HIPCK(hipStreamWaitEvent(B2, S.gx_meta, 0));
        gx.part = 2;
        gx_mark(ctx, seq, kP0, B2);
        HIPCK(launch_store_place(P, S.d_blocks, S.d_bst, S.d_off, S.d_flags, S.d_pre, S.d_rstate, S.d_ev, S.d_slot,
                                 ctx->d_scratch[si], ctx->d_arena, S.d_pcid, S.d_ppos, gx, B2));
        gx_mark(ctx, seq, kP1, B2);
        HIPCK(hipEventRecord(S.placed, B2));
        S.gx_split = true;
    }
    ctx->gx_place_pending = true;
    return 0;
}

// Wait for the placement's read-back: this rank's X3 send counts (send_counts[G]), the checks of
// the allocator scan and of the X3 counts, and the host bookkeeping of the batch.
extern "C" int hdrf_gx_place_wait(hdrf_ctx *ctx, int64_t *send_counts)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 3)) return rc;
    if (!ctx->gx_place_pending) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_place_wait: no placement launched");
    if (!send_counts) return set_err(ctx, HDRF_E_INVAL, "null counts");
    const int si = gx_back_si(ctx);
    Slot &S = ctx->sl[si];
    GxHost *h = S.h_gx;
    HIPCK(hipEventSynchronize(S.gx_meta));
    ctx->gx_place_pending = false;
    if (h->commit_err) {                               // an earlier batch's commit (not waited for)
        HIPCK(hipMemsetAsync(ctx->d_gx_err, 0, sizeof(int), ctx->stB));
        HIPCK(hipStreamSynchronize(ctx->stB));
        const int e = h->commit_err;
        h->commit_err = 0;
        return device_error(ctx, e);
    }
    if (ctx->gx_dscan) {
        ctx->gx_ain = h->st[0];
        ctx->gx_aout = h->st[3];
        if (!*S.h_err && std::memcmp(&h->st[3], &h->st[1], sizeof(AllocState)) != 0)
            return set_err(ctx, HDRF_E_DEVICE, "device allocator scan disagrees with this rank's flush walk");
    } else if (ctx->gx_scanned) {
        if (std::memcmp(&h->st[3], &ctx->gx_expect, sizeof(AllocState)) != 0)
            return set_err(ctx, HDRF_E_DEVICE, "allocator scan disagrees with this rank's flush walk");
    }
    ctx->gx_scanned = 0;
    ctx->gx_dscan = 0;
    if (S.gen_reset && !*S.h_err) {                    // the fresh generation's host side (hdrf_reset_async)
        reset_host(ctx);
        ctx->h_alloc = initial_alloc(ctx);
        S.gen_reset = false;
    }
    // (checked before any host bookkeeping: a failed placement leaves the host state untouched; a
    // device error is complete_slot's to report)
    for (int d = 0; d < ctx->G && !*S.h_err; d++)
        if (h->c3[d] != h->x3want[d])
            return set_err(ctx, HDRF_E_DEVICE, "X3 send count to rank " + std::to_string(d) + " (" +
                                                   std::to_string(h->c3[d]) + ") disagrees with its X2 answers (" +
                                                   std::to_string(h->x3want[d]) + ")");
    // the open containers this rank's flush walk started and ended in hold its placed chunks even
    // when another rank closes them (the node read, hdrf_gx_read_fill, gathers from them)
    for (const AllocState *a : {&ctx->gx_ain, &ctx->gx_aout})
        for (int t = 0; t < ctx->cfg.n_thread; t++)
            if (a->exists[t] && !ctx->containers.count(a->id[t])) note_container(ctx, a->id[t], a->slot[t], a->cur[t], 0);
    S.gx_compressed = false;
    if (int rc = complete_slot(ctx, si, false)) return rc;
    for (int d = 0; d < ctx->G; d++) send_counts[d] = (int64_t)h->c3[d];
    ctx->gx_x3recv.assign(h->x3e, h->x3e + ctx->G);
    ctx->gx_bphase = 4;
    gx_collect(ctx, false, ctx->gx_nback);
    return 0;
}

extern "C" int hdrf_gx_place(hdrf_ctx *ctx, const uint8_t *alloc_final, uint32_t *x3_send, int64_t *send_counts)
{
    HDRF_LOCK(ctx);
    if (!send_counts) return ctx ? set_err(ctx, HDRF_E_INVAL, "null exchange buffer") : HDRF_E_INVAL;
    if (int rc = hdrf_gx_place_launch(ctx, alloc_final, x3_send)) return rc;
    return hdrf_gx_place_wait(ctx, send_counts);
}

// The X3 receive counts this owner's decisions imply (valid from hdrf_gx_place to hdrf_gx_commit):
// the X3 exchange needs no count exchange of its own.
extern "C" int hdrf_gx_x3_counts(hdrf_ctx *ctx, int64_t *recv_counts)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 4)) return rc;
    if (!recv_counts) return set_err(ctx, HDRF_E_INVAL, "null counts");
    for (int s = 0; s < ctx->G; s++) recv_counts[s] = ctx->gx_x3recv[(size_t)s];
    return 0;
}

// ---- node-global compressor 2 (DN/DataDeduplicator.java:748-797: a closing container is rewritten
// as one Lz4Codec file).  A node-global container's bytes lie on the ranks that placed into it (rank
// r continues the container rank r - 1 left open, in the same arena slot index), so the rank whose
// flush walk closes a container first gathers the head pieces the earlier ranks hold
// (hdrf_gx_piece, planned on the host from every rank's hdrf_gx_alloc_io), then compresses the
// containers it closed (hdrf_gx_compress), all between hdrf_gx_place and hdrf_gx_commit.
extern "C" int hdrf_gx_alloc_io(hdrf_ctx *ctx, uint8_t *alloc_in, uint8_t *alloc_out)
{
    HDRF_LOCK(ctx);
    if (!ctx || ctx->G < 2 || !alloc_in || !alloc_out) return ctx ? set_err(ctx, HDRF_E_INVAL, "bad arguments") : HDRF_E_INVAL;
    if (ctx->gx_bphase != 4 && !(ctx->gx_bphase == 3 && !ctx->gx_place_pending && !ctx->gx_dscan))
        return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_alloc_io after hdrf_gx_flush (or hdrf_gx_place with the device scan)");
    std::memset(alloc_in, 0, HDRF_ALLOC_STATE_BYTES);
    std::memcpy(alloc_in, &ctx->gx_ain, sizeof(AllocState));
    std::memset(alloc_out, 0, HDRF_ALLOC_STATE_BYTES);
    std::memcpy(alloc_out, &ctx->gx_aout, sizeof(AllocState));
    return 0;
}

extern "C" int hdrf_gx_piece(hdrf_ctx *ctx, uint32_t id, uint64_t off, uint64_t n, void *dev, int32_t write)
{
    HDRF_LOCK(ctx);
    if (!ctx || ctx->G < 2 || (n && !dev)) return ctx ? set_err(ctx, HDRF_E_INVAL, "bad arguments") : HDRF_E_INVAL;
    if (write && ctx->cfg.compressor != 2)
        return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_piece: writes are the compressor-2 head-piece gather only");
    auto it = ctx->containers.find(id);
    if (it == ctx->containers.end()) return set_err(ctx, HDRF_E_NOTFOUND, "container not resident on this rank");
    if (off > ctx->cfg.container_max || n > ctx->cfg.container_max - off) return set_err(ctx, HDRF_E_INVAL, "piece outside the container");
    uint8_t *p = ctx->d_arena + (size_t)it->second.slot * ctx->cfg.container_max + off;
    if (n) {
        // (an arena copy of this rank's place on stream B2 must have landed before a read)
        for (auto &S : ctx->sl)
            if (S.gx_inuse && S.gx_split) HIPCK(hipStreamWaitEvent(ctx->stB, S.placed, 0));
        HIPCK(hipMemcpyAsync(write ? (void *)p : dev, write ? (const void *)dev : (const void *)p, n, hipMemcpyDeviceToDevice,
                             ctx->stB));
        // a read hands the bytes to the caller (who ships them to the closer): complete on return; a
        // write is ordered before hdrf_gx_compress on the same stream, which synchronises
        if (!write) HIPCK(hipStreamSynchronize(ctx->stB));
    }
    return 0;
}

extern "C" int hdrf_gx_compress(hdrf_ctx *ctx)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    // every return path leaves the queued hdrf_gx_piece writes complete (their source buffers may be
    // released by the caller as soon as this returns)
    if (int rc = gx_check(ctx, 4)) {
        if (ctx->stB) (void)hipStreamSynchronize(ctx->stB);
        return rc;
    }
    const hdrf_cfg &c = ctx->cfg;
    if (c.compressor != 2) {
        HIPCK(hipStreamSynchronize(ctx->stB));
        return 0;
    }
    Slot &S = gx_back_slot(ctx);
    const uint32_t nclosed = *S.h_nclosed;
    if (!nclosed || S.gx_compressed) {                  // once per batch: a second call changes nothing
        HIPCK(hipStreamSynchronize(ctx->stB));         // (hdrf_gx_piece writes are complete on return)
        return 0;
    }
    hipStream_t st = ctx->stB;
    HIPCK(launch_lz4(S.d_closed, S.d_nclosed, ctx->closed_cap, c.container_max, ctx->d_arena, ctx->d_carena, ctx->cslot,
                     S.d_segclen, S.d_filelen, S.d_lzwork, st));
    HIPCK(hipMemcpyAsync(S.h_filelen, S.d_filelen, sizeof(uint32_t) * nclosed, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < nclosed; i++) {
        const ClosedRec &r = S.h_closed[i];
        auto it = ctx->containers.find(r.id);
        if (it == ctx->containers.end()) return set_err(ctx, HDRF_E_DEVICE, "closed container missing");
        it->second.clen = S.h_filelen[i];
        ctx->stats.closed_file_bytes += (int64_t)S.h_filelen[i] - (int64_t)r.len;
    }
    S.gx_compressed = true;
    return (int)nclosed;
}

// The owners' commit of the X3 locations: enqueued on the back stream and not waited for (an
// error it raises is reported by the next hdrf_gx_place or by hdrf_gx_sync).
extern "C" int hdrf_gx_commit(hdrf_ctx *ctx, const uint32_t *x3_recv, const int64_t *recv_counts)
{
    HDRF_LOCK(ctx);
    if (int rc = gx_check(ctx, 4)) return rc;
    if (!x3_recv || !recv_counts) return set_err(ctx, HDRF_E_INVAL, "null exchange buffer");
    for (int s = 0; s < ctx->G; s++) {
        if (recv_counts[s] < 0 || recv_counts[s] > ctx->gx_cap) return set_err(ctx, HDRF_E_INVAL, "bad receive count");
        if (recv_counts[s] != ctx->gx_x3recv[(size_t)s])
            return set_err(ctx, HDRF_E_DEVICE, "X3 receive count from rank " + std::to_string(s) +
                                                   " disagrees with this owner's decisions");
    }
    Slot &S = gx_back_slot(ctx);
    // compressor 2: the containers this rank closed must be Lz4Codec files before the batch commits
    // (container reads of closed containers take their bytes from the compressed arena)
    if (ctx->cfg.compressor == 2 && *S.h_nclosed && !S.gx_compressed)
        return set_err(ctx, HDRF_E_INVAL, "compressor 2: hdrf_gx_compress must run between hdrf_gx_place and hdrf_gx_commit");
    hipStream_t st = ctx->stB;
    const uint64_t seq = ctx->gx_nback;
    std::memcpy(S.h_gx->up_r3, recv_counts, sizeof(int64_t) * ctx->G);
    gx_mark(ctx, seq, kG12, st);
    HIPCK(hipMemcpyAsync(ctx->d_gx_rcounts, S.h_gx->up_r3, sizeof(int64_t) * ctx->G, hipMemcpyHostToDevice, st));
    HIPCK(launch_gx_commit(x3_recv, ctx->d_gx_rcounts, max_count(recv_counts, ctx->G), ctx->gx_cap, ctx->G, ctx->d_tab,
                           ctx->cfg.index_log2, ctx->d_gx_err, st));
    gx_mark(ctx, seq, kG13, st);
    HIPCK(hipEventRecord(S.back_done, st));
    ctx->gx_bphase = 0;
    ctx->gx_nback++;
    return 0;
}

// Complete every node-global batch in flight (all streams) and report an error of the last commits.
static int gx_sync_locked(hdrf_ctx *ctx)
{
    if (int rc = drain(ctx)) return rc;
    int herr = 0;
    HIPCK(hipMemcpy(&herr, ctx->d_gx_err, sizeof(int), hipMemcpyDeviceToHost));
    gx_collect(ctx, true, ctx->gx_nback);
    if (herr) {
        HIPCK(hipMemset(ctx->d_gx_err, 0, sizeof(int)));
        return device_error(ctx, herr);
    }
    return 0;
}

extern "C" int hdrf_gx_sync(hdrf_ctx *ctx)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G < 2) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_* needs cfg.n_ranks > 1");
    return gx_sync_locked(ctx);
}

static int check_b(hdrf_ctx *ctx, int32_t b)
{
    if (!ctx) return HDRF_E_INVAL;
    if (b < 0 || b >= ctx->last_nblocks) return set_err(ctx, HDRF_E_INVAL, "block index out of range");
    return 0;
}

extern "C" int hdrf_batch_info(hdrf_ctx *ctx, int32_t b, int64_t *n_chunks, int64_t *store_size)
{
    HDRF_LOCK(ctx);
    if (int rc = check_b(ctx, b)) return rc;
    const Slot &R = ctx->sl[ctx->res];
    if (n_chunks) *n_chunks = R.h_bst[b].n_chunks;
    if (store_size) *store_size = (int64_t)R.h_store[b];
    return 0;
}

extern "C" int hdrf_batch_offsets(hdrf_ctx *ctx, int32_t b, uint32_t *out, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (int rc = check_b(ctx, b)) return rc;
    const Slot &R = ctx->sl[ctx->res];
    const int64_t n = R.h_bst[b].n_chunks;
    if (cap < n) return set_err(ctx, HDRF_E_CAPACITY, "offsets capacity");
    HIPCK(hipMemcpy(out, R.d_off + (size_t)b * ctx->cap_blk, n * 4, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int hdrf_batch_digests(hdrf_ctx *ctx, int32_t b, uint8_t *out, int64_t cap_bytes)
{
    HDRF_LOCK(ctx);
    if (int rc = check_b(ctx, b)) return rc;
    const Slot &R = ctx->sl[ctx->res];
    const int64_t n = R.h_bst[b].n_chunks;
    if (cap_bytes < n * ctx->H) return set_err(ctx, HDRF_E_CAPACITY, "digest capacity");
    HIPCK(hipMemcpy(out, R.d_dig + (size_t)b * ctx->cap_blk * ctx->HW, n * ctx->H, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int hdrf_batch_is_new(hdrf_ctx *ctx, int32_t b, uint8_t *out, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (int rc = check_b(ctx, b)) return rc;
    const Slot &R = ctx->sl[ctx->res];
    const int64_t n = R.h_bst[b].n_chunks;
    if (cap < n) return set_err(ctx, HDRF_E_CAPACITY, "is_new capacity");
    HIPCK(hipMemcpy(out, R.d_flags + (size_t)b * ctx->cap_blk, n, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; i++) out[i] &= 1;
    return 0;
}

extern "C" int hdrf_batch_placement(hdrf_ctx *ctx, int32_t b, uint32_t *cid, uint32_t *pos, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (int rc = check_b(ctx, b)) return rc;
    const Slot &R = ctx->sl[ctx->res];
    const int64_t n = R.h_bst[b].n_chunks;
    if (cap < n) return set_err(ctx, HDRF_E_CAPACITY, "placement capacity");
    std::vector<uint8_t> f(n);
    HIPCK(hipMemcpy(f.data(), R.d_flags + (size_t)b * ctx->cap_blk, n, hipMemcpyDeviceToHost));
    if (cid) HIPCK(hipMemcpy(cid, R.d_pcid + (size_t)b * ctx->cap_blk, n * 4, hipMemcpyDeviceToHost));
    if (pos) HIPCK(hipMemcpy(pos, R.d_ppos + (size_t)b * ctx->cap_blk, n * 4, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < n; i++)
        if (!(f[i] & 1)) {
            if (cid) cid[i] = 0;
            if (pos) pos[i] = 0;
        }
    return 0;
}

extern "C" int hdrf_reduce_block(hdrf_ctx *ctx, uint64_t block_id, const uint8_t *data, uint64_t len,
                                 hdrf_block_result *out)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G > 1) return set_err(ctx, HDRF_E_INVAL, "node-global context: use the hdrf_gx_* phases");
    if ((int64_t)len > ctx->cfg.max_block_bytes) return set_err(ctx, HDRF_E_INVAL, "block larger than max_block_bytes");
    if (len && !data) return set_err(ctx, HDRF_E_INVAL, "null data");
    const uint64_t need = len + 4096;
    if (ctx->stage_cap < need) {
        if (ctx->d_stage) (void)hipFree(ctx->d_stage);
        ctx->d_stage = nullptr;
        ctx->stage_cap = 0;
        const uint64_t cap = std::max<uint64_t>(need, (uint64_t)ctx->cfg.max_block_bytes + 4096);
        HIPCK(hipMalloc((void **)&ctx->d_stage, cap));
        ctx->stage_cap = cap;
    }
    if (len) HIPCK(hipMemcpyAsync(ctx->d_stage, data, len, hipMemcpyHostToDevice, ctx->st));
    HIPCK(hipMemsetAsync(ctx->d_stage + len, 0, 64, ctx->st));
    const uint8_t *p = ctx->d_stage;
    const uint64_t readable = ctx->stage_cap;
    int rc = hdrf_reduce_batch(ctx, 1, &p, &len, &readable, &block_id);
    if (rc) return rc;
    if (out) {
        int64_t n = 0, ss = 0;
        hdrf_batch_info(ctx, 0, &n, &ss);
        out->n_chunks = n;
        out->store_size = ss;
        if (out->capacity < n && (out->offsets || out->digests || out->is_new || out->container_id || out->container_pos))
            return set_err(ctx, HDRF_E_CAPACITY, "result capacity too small");
        if (out->offsets && (rc = hdrf_batch_offsets(ctx, 0, out->offsets, out->capacity))) return rc;
        if (out->digests && (rc = hdrf_batch_digests(ctx, 0, out->digests, out->capacity * ctx->H))) return rc;
        if (out->is_new && (rc = hdrf_batch_is_new(ctx, 0, out->is_new, out->capacity))) return rc;
        if ((out->container_id || out->container_pos) &&
            (rc = hdrf_batch_placement(ctx, 0, out->container_id, out->container_pos, out->capacity)))
            return rc;
    }
    return 0;
}

// ---- index views ------------------------------------------------------------------------
static void encode_value(const IndexEntry &e, uint8_t v[11])
{
    // chunkMeta.getMeta — DN/chunkMeta.java:62-77
    v[0] = (uint8_t)e.ncopy;
    v[1] = (uint8_t)(e.cid >> 16); v[2] = (uint8_t)(e.cid >> 8); v[3] = (uint8_t)e.cid;
    v[4] = (uint8_t)(e.start >> 16); v[5] = (uint8_t)(e.start >> 8); v[6] = (uint8_t)e.start;
    v[7] = (uint8_t)(e.stop >> 16); v[8] = (uint8_t)(e.stop >> 8); v[9] = (uint8_t)e.stop;
    v[10] = (uint8_t)(((e.start >> 20) & 0xF0) | ((e.stop >> 24) & 0x0F));
}

static void entry_digest(const IndexEntry &e, int H, uint8_t *out)
{
    if (H == 20) {                                   // SHA-1: bytes 0..7 kept in dig[3..4]
        std::memcpy(out, &e.dig[3], 8);
    } else {                                         // SHA-224: bytes 0..6 in the tag, 7 in ncopy
        const unsigned long long t = e.tag & kTag56;
        std::memcpy(out, &t, 7);
        out[7] = (uint8_t)(e.ncopy >> 8);
    }
    std::memcpy(out + 8, e.dig, H == 20 ? 12 : H - 8);
}

extern "C" int hdrf_index_get(hdrf_ctx *ctx, const uint8_t *digest, uint8_t out11[11])
{
    HDRF_LOCK(ctx);
    if (!ctx || !digest) return HDRF_E_INVAL;
    uint32_t dw[2];
    std::memcpy(dw, digest, 8);
    const unsigned long long key = tag_mask(ctx), tag = tag_word(dw, key);
    const uint64_t mask = (1ull << ctx->cfg.index_log2) - 1;
    uint64_t h = tag_home(tag, ctx->cfg.index_log2);
    if (int rc = drain(ctx)) return rc;
    for (uint64_t probe = 0; probe <= mask; probe++) {
        IndexEntry e;
        HIPCK(hipMemcpy(&e, ctx->d_tab + h, sizeof e, hipMemcpyDeviceToHost));
        if (!tag_live(e.tag, key)) return 0;
        uint8_t full[28];
        entry_digest(e, ctx->H, full);
        if (e.tag == tag && std::memcmp(full, digest, ctx->H) == 0) {
            if (out11) encode_value(e, out11);
            return 1;
        }
        h = (h + 1) & mask;
    }
    return 0;
}

static int fetch_table(hdrf_ctx *ctx, std::vector<IndexEntry> &tab)
{
    tab.resize((size_t)1 << ctx->cfg.index_log2);
    if (int rc = drain(ctx)) return rc;
    HIPCK(hipMemcpy(tab.data(), ctx->d_tab, tab.size() * sizeof(IndexEntry), hipMemcpyDeviceToHost));
    return 0;
}

// Probe lengths of the last completed batch (linear probing from each chunk's home slot to the
// entry it resolved to): sum, max and the number of chunks.  Steady-state index measurement.
extern "C" int hdrf_probe_stats(hdrf_ctx *ctx, int64_t *probe_sum, int64_t *probe_max, int64_t *chunks)
{
    HDRF_LOCK(ctx);
    if (!ctx || !probe_sum || !probe_max || !chunks) return HDRF_E_INVAL;
    if (ctx->G > 1) return set_err(ctx, HDRF_E_UNSUPPORTED, "probe stats on node-global contexts");
    if (int rc = drain(ctx)) return rc;
    Slot &S = ctx->sl[ctx->res];
    if (ctx->last_nblocks < 1) return set_err(ctx, HDRF_E_INVAL, "no completed batch");
    unsigned long long *d = nullptr;
    HIPCK(hipMalloc((void **)&d, 3 * sizeof(unsigned long long)));
    unsigned long long h[3] = {0, 0, 0};
    hipError_t e = hipMemsetAsync(d, 0, sizeof h, ctx->st);
    if (e == hipSuccess)
        e = launch_index_probe(ctx->cfg.hasher, S.d_bst, ctx->last_nblocks, ctx->cap_blk, S.d_dig, S.d_slot,
                               ctx->cfg.index_log2, tag_mask(ctx), d, ctx->st);
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, ctx->st);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->st);
    (void)hipFree(d);
    if (e != hipSuccess) return set_err(ctx, HDRF_E_HIP, hipGetErrorString(e));
    *probe_sum = (int64_t)h[0];
    *probe_max = (int64_t)h[1];
    *chunks = (int64_t)h[2];
    return 0;
}

extern "C" int64_t hdrf_index_count(hdrf_ctx *ctx)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    std::vector<IndexEntry> tab;
    if (int rc = fetch_table(ctx, tab)) return rc;
    int64_t n = 0;
    const unsigned long long key = tag_mask(ctx);
    for (auto &e : tab) n += tag_live(e.tag, key);
    return n;
}

extern "C" int64_t hdrf_index_dump(hdrf_ctx *ctx, uint8_t *keys, uint8_t *vals, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    std::vector<IndexEntry> tab;
    if (int rc = fetch_table(ctx, tab)) return rc;
    const int H = ctx->H;
    std::vector<std::vector<uint8_t>> rows;
    const unsigned long long key = tag_mask(ctx);
    for (auto &e : tab) {
        if (!tag_live(e.tag, key)) continue;
        std::vector<uint8_t> r(H + 11);
        entry_digest(e, H, r.data());
        encode_value(e, r.data() + H);
        rows.push_back(std::move(r));
    }
    if ((int64_t)rows.size() > cap) return set_err(ctx, HDRF_E_CAPACITY, "index dump capacity");
    std::sort(rows.begin(), rows.end(),
              [H](const std::vector<uint8_t> &a, const std::vector<uint8_t> &b) { return std::memcmp(a.data(), b.data(), H) < 0; });
    for (size_t i = 0; i < rows.size(); i++) {
        std::memcpy(keys + i * H, rows[i].data(), H);
        std::memcpy(vals + i * 11, rows[i].data() + H, 11);
    }
    return (int64_t)rows.size();
}

extern "C" int hdrf_allocator(hdrf_ctx *ctx, uint8_t out24[24])
{
    HDRF_LOCK(ctx);
    if (!ctx || !out24) return HDRF_E_INVAL;
    if (!ctx->have_alloc) return 0;
    uint32_t v[8];
    for (int t = 0; t < 4; t++) {
        v[t] = ctx->h_alloc.id[t];
        v[t + 4] = ctx->h_alloc.pos[t];
    }
    for (int i = 0; i < 8; i++) {                   // utilities.blockIDtoBytes (DN/utilities.java:66-75)
        out24[3 * i] = (uint8_t)(v[i] >> 16);
        out24[3 * i + 1] = (uint8_t)(v[i] >> 8);
        out24[3 * i + 2] = (uint8_t)v[i];
    }
    return 1;
}

// ---- restore (index persistence: a DataNode restarting on its Redis dump + chunkDir) -------
// SET digest -> value for n entries (the rows of hdrf_index_dump) on a context whose index does
// not hold these digests yet (a fresh or reset context).
extern "C" int hdrf_index_load(hdrf_ctx *ctx, const uint8_t *keys, const uint8_t *vals, int64_t n)
{
    HDRF_LOCK(ctx);
    if (!ctx || n < 0 || (n && (!keys || !vals))) return HDRF_E_INVAL;
    if (ctx->G > 1) return set_err(ctx, HDRF_E_UNSUPPORTED, "restore on node-global contexts: not yet");
    if (int rc = drain(ctx)) return rc;
    if (n == 0) return 0;
    const uint64_t o_dw = 0, dw_b = (uint64_t)n * ctx->HW * 4;
    const uint64_t o_v = (dw_b + 255) & ~255ull, o_err = (o_v + (uint64_t)n * 11 + 255) & ~255ull;
    if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, o_err + 256)) return rc;
    uint8_t *R = ctx->d_rd;
    hipStream_t st = ctx->st;
    std::vector<uint8_t> dw(dw_b, 0);                  // digest bytes as u32 words (SHA-224: 28 B)
    for (int64_t k = 0; k < n; k++) std::memcpy(dw.data() + (size_t)k * ctx->HW * 4, keys + (size_t)k * ctx->H, ctx->H);
    HIPCK(hipMemcpyAsync(R + o_dw, dw.data(), dw_b, hipMemcpyHostToDevice, st));
    HIPCK(hipMemcpyAsync(R + o_v, vals, (size_t)n * 11, hipMemcpyHostToDevice, st));
    HIPCK(hipMemsetAsync(R + o_err, 0, 4, st));
    HIPCK(launch_index_load(ctx->cfg.hasher, (const uint32_t *)(R + o_dw), R + o_v, (int)n, ctx->d_tab,
                            ctx->cfg.index_log2, tag_mask(ctx), ++ctx->batch, (int *)(R + o_err), st));
    int err = 0;
    HIPCK(hipMemcpyAsync(&err, R + o_err, 4, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    if (err) return set_err(ctx, HDRF_E_CAPACITY, "index table full (index_log2 too small)");
    return 0;
}

// SET "blockID" (the 24-B allocator, DN/utilities.java:66-75) and reopen the three storer
// ranges' open containers from their chunkDir files (open_len[t] < 0: no file): the storer
// appends to them exactly as threadedStorer does after reading prevData (:723-737).
extern "C" int hdrf_allocator_load(hdrf_ctx *ctx, const uint8_t alloc24[24], const uint8_t *const *open_files,
                                   const int64_t *open_len)
{
    HDRF_LOCK(ctx);
    if (!ctx || !alloc24 || !open_len) return HDRF_E_INVAL;
    if (ctx->G > 1) return set_err(ctx, HDRF_E_UNSUPPORTED, "restore on node-global contexts: not yet");
    if (int rc = drain(ctx)) return rc;
    AllocState a{};
    for (int i = 0; i < 8; i++) {
        const uint32_t v = ((uint32_t)alloc24[3 * i] << 16) | ((uint32_t)alloc24[3 * i + 1] << 8) | alloc24[3 * i + 2];
        if (i < 4) a.id[i] = v; else a.pos[i - 4] = v;
    }
    for (int t = 0; t < 4; t++) a.slot[t] = (uint32_t)t * (uint32_t)(ctx->cfg.arena_slots / 4);
    for (int t = 0; t < ctx->cfg.n_thread; t++) {
        if (open_len[t] < 0) continue;
        if ((uint64_t)open_len[t] > ctx->cfg.container_max || (open_len[t] && (!open_files || !open_files[t])))
            return set_err(ctx, HDRF_E_INVAL, "bad open container file");
        if (open_len[t])
            HIPCK(hipMemcpy(ctx->d_arena + (size_t)a.slot[t] * ctx->cfg.container_max, open_files[t],
                            (size_t)open_len[t], hipMemcpyHostToDevice));
        a.cur[t] = (uint32_t)open_len[t];
        a.exists[t] = 1;
    }
    HIPCK(hipMemcpy(ctx->d_alloc, &a, sizeof a, hipMemcpyHostToDevice));
    ctx->h_alloc = a;
    ctx->have_alloc = 1;
    for (int t = 0; t < ctx->cfg.n_thread; t++)
        if (a.exists[t]) note_container(ctx, a.id[t], a.slot[t], a.cur[t], 0);
    return 0;
}

// SET longToBytes(blockId,4) -> recipe (storeDB, DN/DataDeduplicator.java:372-392)
extern "C" int hdrf_recipe_load(hdrf_ctx *ctx, uint64_t block_id, const uint8_t *recipe, int64_t len)
{
    HDRF_LOCK(ctx);
    if (!ctx || !recipe || len < 4 || (len - 4) % ctx->H) return HDRF_E_INVAL;
    const uint32_t key = (uint32_t)block_id;
    if (int rc = drain(ctx)) return rc;
    const uint32_t n = (uint32_t)((len - 4) / ctx->H);
    uint8_t *dst = nullptr;
    if (int rc = recipe_alloc(ctx, (uint64_t)n * ctx->H, key, n, &dst)) return rc;
    if (n) HIPCK(hipMemcpy(dst, recipe + 4, (size_t)n * ctx->H, hipMemcpyHostToDevice));
    ctx->lengths[key] = ((int64_t)recipe[0] << 24) | (recipe[1] << 16) | (recipe[2] << 8) | recipe[3];
    return 0;
}

extern "C" int64_t hdrf_recipe_get(hdrf_ctx *ctx, uint64_t block_id, uint8_t *out, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (int rc = drain(ctx)) return rc;                 // blocks in flight first: their recipes are SET
    auto it = ctx->recipes.find((uint32_t)block_id);
    if (it == ctx->recipes.end()) return 0;
    const int64_t n = 4 + (int64_t)it->second.n * ctx->H;
    if (!out || cap < n) return set_err(ctx, HDRF_E_CAPACITY, "recipe needs " + std::to_string(n) + " bytes");
    std::vector<uint8_t> r;
    const int fr = fetch_recipe(ctx, (uint32_t)block_id, r);
    if (fr < 0) return fr;
    std::memcpy(out, r.data(), (size_t)n);
    return n;
}

extern "C" int64_t hdrf_block_length(hdrf_ctx *ctx, uint64_t block_id)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    auto it = ctx->lengths.find((uint32_t)block_id);
    return it == ctx->lengths.end() ? HDRF_E_NOTFOUND : it->second;
}

extern "C" int64_t hdrf_container_read(hdrf_ctx *ctx, uint32_t id, uint8_t *out, int64_t cap, int32_t *closed)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (int rc = drain(ctx)) return rc;                 // batches in flight may append, close or recycle it
    auto it = ctx->containers.find(id);
    if (it == ctx->containers.end()) return set_err(ctx, HDRF_E_NOTFOUND, "container not resident");
    if (closed) *closed = it->second.closed;
    const bool lz = ctx->cfg.compressor == 2 && it->second.closed;     // the file is the Lz4Codec stream
    const int64_t n = lz ? it->second.clen : it->second.len;
    if (!out) return n;
    if (cap < n) return set_err(ctx, HDRF_E_CAPACITY, "container capacity");
    const uint8_t *src = lz ? ctx->d_carena + (size_t)it->second.slot * ctx->cslot
                            : ctx->d_arena + (size_t)it->second.slot * ctx->cfg.container_max;
    if (n) HIPCK(hipMemcpy(out, src, n, hipMemcpyDeviceToHost));
    return n;
}

// ---- durable containers: the chunkDir files of the storers (DN/DataDeduplicator.java:748-818) ----
// Since the last drain: every container that closed (the whole file: raw bytes, or the Lz4Codec
// stream under compressor 2, rewritten at :748-786) in close order, then every open container's
// bytes appended since (:806-818).  Events are emitted whole, in order, while they fit.  Only what
// the COMPLETED batches (hdrf_wait_batch) produced is handed out; batches still in flight keep
// running: their place kernels only append past the bytes copied here, and a closed container's
// slot stays retained until it is drained.  The D2H copies run on stream D, so they overlap the
// H2D copies of later batches on stream C (PCIe is full duplex).
extern "C" int64_t hdrf_drain_containers(hdrf_ctx *ctx, hdrf_container_event *ev, int64_t ev_cap, uint8_t *out,
                                         int64_t out_cap, int64_t *need)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (need) *need = 0;
    if (!ctx->cfg.retain_containers) return set_err(ctx, HDRF_E_INVAL, "hdrf_drain_containers needs cfg.retain_containers");
    if (ctx->G > 1) return set_err(ctx, HDRF_E_UNSUPPORTED, "container drain on node-global contexts");
    if (ev_cap < 0 || out_cap < 0 || (ev_cap && !ev) || (out_cap && !out)) return set_err(ctx, HDRF_E_INVAL, "bad buffers");
    const hdrf_cfg &c = ctx->cfg;
    struct Pend { uint32_t id; int closed; int64_t off, n; ContainerInfo ci; };
    std::vector<Pend> todo;
    for (uint32_t id : ctx->pend_closed) {
        auto it = ctx->containers.find(id);
        if (it == ctx->containers.end()) return set_err(ctx, HDRF_E_DEVICE, "undrained container missing");
        if (c.compressor == 2) {                          // the whole Lz4Codec file replaces the raw one
            todo.push_back(Pend{id, 1, 0, (int64_t)it->second.clen, it->second});
        } else {
            // the storer's close rewrites the file as prevData || buffer (:754-786): the bytes already
            // handed out plus the rest, so only the rest travels (file_off = the bytes handed out)
            const int64_t done = ctx->handed.count(id) ? ctx->handed[id] : 0;
            todo.push_back(Pend{id, 1, done, (int64_t)it->second.len - done, it->second});
        }
    }
    const size_t nclosed = todo.size();
    for (int t = 0; t < c.n_thread; t++) {
        if (!ctx->h_alloc.exists[t]) continue;
        const uint32_t id = ctx->h_alloc.id[t];
        auto it = ctx->containers.find(id);
        if (it == ctx->containers.end()) continue;
        const int64_t done = ctx->handed.count(id) ? ctx->handed[id] : 0;
        if ((int64_t)it->second.len > done) todo.push_back(Pend{id, 0, done, (int64_t)it->second.len - done, it->second});
    }
    // pinned (device-mapped) output: the CUs write it (xfer_kernel), beside the SDMA H2D of later
    // batches (whole blocks through hdrf_submit_host: 38.8 / 39.1 vs 34.7 / 35.5 GB/s with the copy
    // engine); once the context receives packets (hdrf_rx_begin), the copy engine (22.0 vs 28.3 GB/s
    // for 64 KiB packets, profiles/r03_c5_drain_ab.txt); pageable output: hipMemcpyAsync.
    // HDRF_DRAIN_KERNEL=1 / 0 forces the CUs / the copy engine.
    static const int kern_env = [] { const char *e = getenv("HDRF_DRAIN_KERNEL"); return e ? (atoi(e) != 0) : -1; }();
    const bool kern = kern_env >= 0 ? kern_env != 0 : !ctx->rx_used;
    hipPointerAttribute_t pa;
    const bool mapped = kern && out_cap > 0 && hipPointerGetAttributes(&pa, out) == hipSuccess &&
                        pa.type == hipMemoryTypeHost && pa.devicePointer != nullptr;
    (void)hipGetLastError();
    if (mapped && ctx->xfer_cap == 0) {
        HIPCK(hipHostMalloc((void **)&ctx->h_xfer, sizeof(XferJob) * 1024, hipHostMallocDefault));
        ctx->xfer_cap = 1024;
    }
    int64_t k = 0, used = 0;
    int nj = 0;
    uint64_t maxj = 0;
    // CU drain grid: one workgroup per ~256 MiB of this drain, at least 5.  Five workgroups still drain
    // a config-5 batch in ~19.5 ms, but the next blocks' H2D copies beside them keep 54.9 GB/s, where
    // a full grid's flood of PCIe writes cut them to 44.6 (config 5 whole blocks: 50.0 / 50.1 GB/s
    // with 5 workgroups, 49.8 / 48.5 with 4, 41.5 with 3, 47.3 / 47.4 with one per item;
    // profiles/r04_drain_wgs_ab.txt, r04_c5_trace3.txt).  HDRF_XFER_WGS = W overrides (0: one per item).
    static const int wgs_env = [] { const char *e = getenv("HDRF_XFER_WGS"); return e ? atoi(e) : -1; }();
    int64_t drain_bytes = 0;
    for (const Pend &e : todo) drain_bytes += e.n;
    const int wgs = wgs_env >= 0 ? wgs_env : (int)std::max<int64_t>(5, (drain_bytes + (256ll << 20) - 1) / (256ll << 20));
    for (const Pend &e : todo) {
        if (k >= ev_cap || used + e.n > out_cap) {
            if (need) *need = e.n;
            break;
        }
        const uint8_t *src = (e.closed && c.compressor == 2) ? ctx->d_carena + (size_t)e.ci.slot * ctx->cslot
                                                             : ctx->d_arena + (size_t)e.ci.slot * c.container_max;
        if (e.n && mapped) {
            if (nj == ctx->xfer_cap) {                    // job list full: flush it
                HIPCK(launch_xfer(ctx->h_xfer, nj, maxj, wgs, ctx->stD));
                HIPCK(hipStreamSynchronize(ctx->stD));
                nj = 0;
                maxj = 0;
            }
            ctx->h_xfer[nj++] = XferJob{(uint64_t)(uintptr_t)(src + e.off),
                                        (uint64_t)(uintptr_t)((uint8_t *)pa.devicePointer + used), (uint64_t)e.n};
            maxj = std::max<uint64_t>(maxj, (uint64_t)e.n);
        } else if (e.n) {
            HIPCK(hipMemcpyAsync(out + used, src + e.off, (size_t)e.n, hipMemcpyDeviceToHost, ctx->stD));
        }
        ev[k] = hdrf_container_event{e.id, e.closed, e.off, e.n, used};
        used += e.n;
        k++;
    }
    if (nj) HIPCK(launch_xfer(ctx->h_xfer, nj, maxj, wgs, ctx->stD));
    HIPCK(hipStreamSynchronize(ctx->stD));
    // the emitted ones are handed over
    const size_t kc = std::min<size_t>((size_t)k, nclosed);
    for (size_t i = 0; i < kc; i++) {
        const uint32_t id = ctx->pend_closed[i];
        ctx->undrained[std::min<uint32_t>(id >> 22, 3)]--;
        ctx->handed.erase(id);
    }
    ctx->pend_closed.erase(ctx->pend_closed.begin(), ctx->pend_closed.begin() + kc);
    for (size_t i = nclosed; i < (size_t)k; i++) ctx->handed[todo[i].id] = todo[i].off + todo[i].n;
    if (k == 0 && !todo.empty()) return set_err(ctx, HDRF_E_CAPACITY, "drain buffer too small for the next event");
    return k;
}

// ---- arrival tickets: the FIFO of DN/DataDeduplicator.java:124-158 (DN/DDRunner.java:20-36) ------
extern "C" int hdrf_ticket_take(hdrf_ctx *ctx, uint64_t *ticket)
{
    HDRF_LOCK(ctx);
    if (!ctx || !ticket) return HDRF_E_INVAL;
    *ticket = ctx->next_ticket++;
    return 0;
}

static void ticket_done(hdrf_ctx *ctx, uint64_t ticket)
{
    if (ctx->serving == ticket) {
        ctx->serving++;
        while (ctx->cancelled.count(ctx->serving)) ctx->cancelled.erase(ctx->serving++);
    } else if (ticket > ctx->serving) {
        ctx->cancelled.insert(ticket);
    }
    ctx->turn.notify_all();
}

extern "C" int hdrf_ticket_cancel(hdrf_ctx *ctx, uint64_t ticket)
{
    HDRF_LOCK(ctx);
    if (!ctx || ticket >= ctx->next_ticket) return HDRF_E_INVAL;
    ticket_done(ctx, ticket);
    return 0;
}

extern "C" int hdrf_reduce_block_ticketed(hdrf_ctx *ctx, uint64_t ticket, uint64_t block_id, const uint8_t *data,
                                          uint64_t len, hdrf_block_result *out)
{
    if (!ctx) return HDRF_E_INVAL;
    std::unique_lock<std::recursive_mutex> lk(ctx->mu);
    if (ticket >= ctx->next_ticket || ticket < ctx->serving || ctx->cancelled.count(ticket))
        return set_err(ctx, HDRF_E_INVAL, "unknown or finished ticket");
    ctx->turn.wait(lk, [&] { return ctx->serving == ticket; });
    const int rc = hdrf_reduce_block(ctx, block_id, data, len, out);
    ticket_done(ctx, ticket);
    return rc;
}

// ---- read side: DataConstructor (DN/DataConstructor.java:73-250, 360-531) --------------------
static int grow(hdrf_ctx *ctx, uint8_t **p, uint64_t *cap, uint64_t need)
{
    if (*cap >= need) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIPCK(hipMalloc((void **)p, need));
    *cap = need;
    return 0;
}

extern "C" int64_t hdrf_reconstruct(hdrf_ctx *ctx, const uint8_t *recipe, int64_t recipe_len, uint8_t *dev_out,
                                    int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx || !recipe || recipe_len < 4) return HDRF_E_INVAL;
    if (ctx->G > 1)
        return set_err(ctx, HDRF_E_UNSUPPORTED, "node-global contexts read through hdrf_gx_read_locate / _fill (every rank)");
    if (int rc = drain(ctx)) return rc;
    const int64_t size = ((int64_t)recipe[0] << 24) | (recipe[1] << 16) | (recipe[2] << 8) | recipe[3];
    const int64_t n = recipe_len / ctx->H;             // t1data.length / hash_length (:223)
    if (size > cap || (size && !dev_out)) return set_err(ctx, HDRF_E_CAPACITY, "output capacity");
    if (n == 0) return size == 0 ? 0 : set_err(ctx, HDRF_E_DEVICE, "recipe without digests");
    // readable containers sorted by id: arena-resident ones, then those loaded back from files
    std::map<uint32_t, uint64_t> rdbl;
    for (auto &kv : ctx->loaded) rdbl[kv.first] = (uint64_t)(uintptr_t)kv.second.ptr;
    for (auto &kv : ctx->containers)
        rdbl[kv.first] = (uint64_t)(uintptr_t)(ctx->d_arena + (size_t)kv.second.slot * ctx->cfg.container_max);
    std::vector<uint32_t> cid;
    std::vector<uint64_t> base;
    for (auto &kv : rdbl) { cid.push_back(kv.first); base.push_back(kv.second); }
    const int ncont = (int)cid.size();
    const uint64_t o_dig = 0, dig_b = (uint64_t)n * ctx->HW * 4;
    const uint64_t o_ch = (dig_b + 255) & ~255ull, ch_b = (uint64_t)n * rd_chunk_bytes();
    const uint64_t o_base = (o_ch + ch_b + 255) & ~255ull, base_b = (uint64_t)std::max(1, ncont) * 8;
    const uint64_t o_cid = (o_base + base_b + 255) & ~255ull, cid_b = (uint64_t)std::max(1, ncont) * 4;
    const uint64_t o_tot = (o_cid + cid_b + 255) & ~255ull;
    if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, o_tot + 256)) return rc;
    uint8_t *R = ctx->d_rd;
    hipStream_t st = ctx->st;
    HIPCK(hipMemcpyAsync(R + o_dig, recipe + 4, (size_t)n * ctx->H, hipMemcpyHostToDevice, st));
    if (ncont) {
        HIPCK(hipMemcpyAsync(R + o_cid, cid.data(), cid.size() * 4, hipMemcpyHostToDevice, st));
        HIPCK(hipMemcpyAsync(R + o_base, base.data(), base.size() * 8, hipMemcpyHostToDevice, st));
    }
    HIPCK(hipMemsetAsync(R + o_tot, 0, 16, st));
    const uint64_t *bases = (const uint64_t *)(R + o_base);
    HIPCK(launch_reconstruct(ctx->cfg.hasher, (const uint32_t *)(R + o_dig), (int)n, ctx->d_tab, ctx->cfg.index_log2,
                             tag_mask(ctx), (const uint32_t *)(R + o_cid), bases, ncont, R + o_ch,
                             (uint64_t *)(R + o_tot), dev_out, (int *)(R + o_tot + 8), st, false));
    uint64_t tot[2] = {0, 0};
    HIPCK(hipMemcpyAsync(tot, R + o_tot, 16, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    if ((int)tot[1]) return set_err(ctx, HDRF_E_NOTFOUND, "a recipe digest or its container is not readable");
    if ((int64_t)tot[0] != size) return set_err(ctx, HDRF_E_DEVICE, "chunk lengths do not add up to the recipe size");
    HIPCK(launch_reconstruct(ctx->cfg.hasher, nullptr, (int)n, nullptr, 0, 0, nullptr, bases, 0, R + o_ch, nullptr,
                             dev_out, nullptr, st, true));
    HIPCK(hipStreamSynchronize(st));
    return size;
}

extern "C" int64_t hdrf_reconstruct_block(hdrf_ctx *ctx, uint64_t block_id, uint8_t *out, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (int rc = drain(ctx)) return rc;
    std::vector<uint8_t> rec;                            // GET longToBytes(blockId,4) (DN/BlockSender.java:292-328)
    const int fr = fetch_recipe(ctx, (uint32_t)block_id, rec);
    if (fr < 0) return fr;
    if (!fr) return set_err(ctx, HDRF_E_NOTFOUND, "no recipe for this block (keep_recipes?)");
    const int64_t size = ((int64_t)rec[0] << 24) | (rec[1] << 16) | (rec[2] << 8) | rec[3];
    if (!out || cap < size) return set_err(ctx, HDRF_E_CAPACITY, "needs " + std::to_string(size) + " bytes");
    if (int rc = grow(ctx, &ctx->d_stage, &ctx->stage_cap, (uint64_t)size + 4096)) return rc;
    const int64_t got = hdrf_reconstruct(ctx, rec.data(), (int64_t)rec.size(), ctx->d_stage, size);
    if (got < 0) return got;
    if (got) HIPCK(hipMemcpy(out, ctx->d_stage, got, hipMemcpyDeviceToHost));
    return got;
}

// ---- node-global read (G > 1): DataConstructor over the node's one index ------------------
// Every rank takes part (include/hdrf.h): the owners locate the digests they own, the locations
// are combined (sum of disjoint rows), and every rank gathers the chunks it placed; the partial
// blocks are disjoint, so their byte sum on the reading rank is the block (hdrf_amd/node.py).
extern "C" int64_t hdrf_gx_read_locate(hdrf_ctx *ctx, const uint8_t *digests, int64_t n, uint32_t *loc)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G < 2) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_read_* needs cfg.n_ranks > 1");
    if (n < 0 || (n && (!digests || !loc))) return set_err(ctx, HDRF_E_INVAL, "bad locate arguments");
    if (n == 0) return 0;
    if (ctx->gx_nfront != ctx->gx_nback) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_read_locate: a batch is in flight");
    // the last batch's commit (stream B) and arena copy (stream B2) land first; a commit error is reported here
    if (int rc = gx_sync_locked(ctx)) return rc;
    const uint64_t o_loc = (((uint64_t)n * ctx->H) + 255) & ~255ull, o_err = o_loc + (((uint64_t)n * 16 + 255) & ~255ull);
    if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, o_err + 256)) return rc;
    uint8_t *R = ctx->d_rd;
    hipStream_t st = ctx->st;
    HIPCK(hipMemcpyAsync(R, digests, (size_t)n * ctx->H, hipMemcpyHostToDevice, st));
    HIPCK(hipMemsetAsync(R + o_err, 0, 4, st));
    HIPCK(launch_gx_locate(ctx->cfg.hasher, (const uint32_t *)R, (int)n, ctx->d_tab, ctx->cfg.index_log2, tag_mask(ctx),
                           ctx->G, ctx->cfg.rank, (uint32_t *)(R + o_loc), (int *)(R + o_err), st));
    int herr = 0;
    HIPCK(hipMemcpyAsync(loc, R + o_loc, (size_t)n * 16, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(&herr, R + o_err, 4, hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    if (herr) return set_err(ctx, HDRF_E_NOTFOUND, "a recipe digest owned by this rank is not in its index partition");
    int64_t mine = 0;
    for (int64_t k = 0; k < n; k++) mine += loc[4 * k + 3] != 0;
    return mine;
}

extern "C" int64_t hdrf_gx_read_fill(hdrf_ctx *ctx, const uint32_t *loc, int64_t n, uint8_t *dev_out, int64_t cap)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (ctx->G < 2) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_read_* needs cfg.n_ranks > 1");
    if (n < 0 || (n && !loc)) return set_err(ctx, HDRF_E_INVAL, "bad fill arguments");
    if (ctx->gx_nfront != ctx->gx_nback) return set_err(ctx, HDRF_E_INVAL, "hdrf_gx_read_fill: a batch is in flight");
    if (int rc = gx_sync_locked(ctx)) return rc;
    struct RdChunkH { uint32_t slot, start, len, off; };
    static_assert(sizeof(RdChunkH) == 16, "RdChunk layout");
    if (rd_chunk_bytes() != sizeof(RdChunkH)) return set_err(ctx, HDRF_E_DEVICE, "RdChunk layout");
    std::vector<RdChunkH> mine;
    std::vector<uint64_t> bases;
    std::map<uint32_t, uint32_t> base_of;               // container id -> index in bases
    uint64_t off = 0, filled = 0;
    for (int64_t k = 0; k < n; k++) {
        const uint32_t *r = loc + 4 * k;
        if (r[3] == 0 || r[2] < r[1]) return set_err(ctx, HDRF_E_INVAL, "location without its placing rank");
        const uint32_t len = r[2] - r[1];
        if ((int)r[3] - 1 == ctx->cfg.rank && len) {
            auto it = ctx->containers.find(r[0]);
            if (it == ctx->containers.end()) return set_err(ctx, HDRF_E_NOTFOUND, "container of a placed chunk is not resident");
            auto b = base_of.find(r[0]);
            if (b == base_of.end()) {
                b = base_of.emplace(r[0], (uint32_t)bases.size()).first;
                bases.push_back((uint64_t)(uintptr_t)(ctx->d_arena + (size_t)it->second.slot * ctx->cfg.container_max));
            }
            if ((uint64_t)r[2] > ctx->cfg.container_max) return set_err(ctx, HDRF_E_DEVICE, "chunk beyond its container");
            mine.push_back(RdChunkH{b->second, r[1], len, (uint32_t)off});
            filled += len;
        }
        off += len;
    }
    if ((int64_t)off > cap || (off && !dev_out)) return set_err(ctx, HDRF_E_CAPACITY, "output capacity");
    if (!mine.empty()) {
        const uint64_t o_b = ((mine.size() * sizeof(RdChunkH)) + 255) & ~255ull;
        if (int rc = grow(ctx, &ctx->d_rd, &ctx->rd_cap, o_b + bases.size() * 8 + 256)) return rc;
        uint8_t *R = ctx->d_rd;
        hipStream_t st = ctx->st;
        HIPCK(hipMemcpyAsync(R, mine.data(), mine.size() * sizeof(RdChunkH), hipMemcpyHostToDevice, st));
        HIPCK(hipMemcpyAsync(R + o_b, bases.data(), bases.size() * 8, hipMemcpyHostToDevice, st));
        HIPCK(launch_rd_gather(R, (int)mine.size(), (const uint64_t *)(R + o_b), dev_out, st));
        HIPCK(hipStreamSynchronize(st));
    }
    return (int64_t)filled;
}

// ---- memory helpers, corpus, timing ------------------------------------------------------
extern "C" int hdrf_dev_alloc(hdrf_ctx *ctx, uint64_t bytes, void **out)
{
    HDRF_LOCK(ctx);
    if (!ctx || !out) return HDRF_E_INVAL;
    HIPCK(hipMalloc(out, bytes));
    return 0;
}

extern "C" int hdrf_dev_free(hdrf_ctx *ctx, void *p)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    if (int rc = drain(ctx)) return rc;
    HIPCK(hipFree(p));
    return 0;
}

extern "C" int hdrf_memcpy_h2d(hdrf_ctx *ctx, void *dst, const void *src, uint64_t bytes)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    HIPCK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, ctx->st));
    HIPCK(hipStreamSynchronize(ctx->st));
    return 0;
}

extern "C" int hdrf_memcpy_d2h(hdrf_ctx *ctx, void *dst, const void *src, uint64_t bytes)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    HIPCK(hipStreamSynchronize(ctx->st));
    HIPCK(hipStreamSynchronize(ctx->stB));
    HIPCK(hipStreamSynchronize(ctx->stB2));
    HIPCK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return 0;
}

extern "C" int hdrf_synchronize(hdrf_ctx *ctx)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    return drain(ctx);                                 // completes every batch in flight
}

extern "C" int hdrf_corpus_fill(hdrf_ctx *ctx, uint8_t *dev, const uint32_t *roots_host, int64_t nblocks,
                                int64_t segs_per_block, int64_t seg_bytes, uint64_t seed)
{
    HDRF_LOCK(ctx);
    return hdrf_corpus_fill_kind(ctx, dev, roots_host, nblocks, segs_per_block, seg_bytes, seed, 0);
}

extern "C" int hdrf_corpus_fill_kind(hdrf_ctx *ctx, uint8_t *dev, const uint32_t *roots_host, int64_t nblocks,
                                     int64_t segs_per_block, int64_t seg_bytes, uint64_t seed, int32_t mixed)
{
    HDRF_LOCK(ctx);
    if (!ctx || !dev || !roots_host || seg_bytes % 16 != 0) return HDRF_E_INVAL;
    uint32_t *d_roots = nullptr;
    const size_t n = (size_t)nblocks * segs_per_block;
    HIPCK(hipMalloc((void **)&d_roots, n * 4));
    HIPCK(hipMemcpyAsync(d_roots, roots_host, n * 4, hipMemcpyHostToDevice, ctx->st));
    HIPCK(launch_corpus(dev, d_roots, nblocks, segs_per_block, seg_bytes, seed, mixed ? 1 : 0, ctx->st));
    HIPCK(hipStreamSynchronize(ctx->st));
    HIPCK(hipFree(d_roots));
    return 0;
}

extern "C" int hdrf_get_stats(hdrf_ctx *ctx, hdrf_stats *out)
{
    HDRF_LOCK(ctx);
    if (!ctx || !out) return HDRF_E_INVAL;
    *out = ctx->stats;
    return 0;
}

extern "C" int hdrf_stage_times(hdrf_ctx *ctx, double *ms, int32_t n, int32_t reset)
{
    HDRF_LOCK(ctx);
    if (!ctx) return HDRF_E_INVAL;
    for (int i = 0; i < n && i < kStages; i++) ms[i] = ctx->stage_ms[i];
    if (reset)
        for (double &v : ctx->stage_ms) v = 0;
    return 0;
}
