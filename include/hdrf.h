/*
 * hdrf.h — C-ABI of libhdrf, the MI355X (gfx950) reduction backend for HDRF's
 * per-block write path (chunk -> fingerprint -> index -> container store).
 *
 * This is the drop-in boundary a DataNode binds through JNI.  Every
 * entry point replaces a piece of the reference's Java path; `DN/` abbreviates
 * hadoop-hdfs/src/main/java/org/apache/hadoop/hdfs/server/datanode/ in /root/reference.
 *
 * Conventions: plain pointers and sizes only; every function returns 0 on success or a
 * negative HDRF_E* code; hdrf_last_error() describes the last failure of a context; no C++
 * exception crosses this ABI.  A context is bound to one GPU.  Threads: every entry point takes
 * the context's lock, so any number of threads (one DataXceiver / DDRunner thread per block) may
 * call it concurrently (hdrf_close excepted: no call may be in progress or follow).  Block ORDER is
 * the call order unless the caller uses arrival tickets (hdrf_ticket_take at block arrival,
 * hdrf_reduce_block_ticketed later from any thread), which reproduce the reference's FIFO
 * (DN/DataDeduplicator.java:124-158, 197-204; DN/DDRunner.java:20-36).  hdrf_last_error() is the
 * context's last error, whichever thread caused it.
 */
#ifndef HDRF_H
#define HDRF_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

#define HDRF_OK 0
#define HDRF_E_INVAL (-1)      /* bad argument / configuration */
#define HDRF_E_HIP (-2)        /* HIP runtime failure */
#define HDRF_E_NOMEM (-3)      /* device or host allocation failed */
#define HDRF_E_CAPACITY (-4)   /* index table, arena or event list full */
#define HDRF_E_NOTFOUND (-5)   /* key / block / container absent */
#define HDRF_E_UNSUPPORTED (-6)/* option not implemented in this build */
#define HDRF_E_DEVICE (-7)     /* a kernel reported an inconsistency */

typedef struct hdrf_ctx hdrf_ctx;

/* Knobs of the reference, all compile-time statics there. */
typedef struct {
    int32_t hasher;          /* 0 SHA-1, 1 SHA-224          DataNode.hasher, DN/DataNode.java:446 */
    int32_t compressor;      /* 1 dedup, 2 dedup + Lz4Codec closed containers   DataNode.compressor :438 */
    int32_t window;          /* 700                         DataDeduplicator.chunking :266 */
    int32_t max_chunk;       /* 1000000                     DataDeduplicator.chunking :272 */
    int32_t n_thread;        /* 3                           DataDeduplicator.nThread :93 */
    int32_t min_mt_chunks;   /* 25                          DataDeduplicator :316, :514 */
    uint32_t container_max;  /* 2^25                        DataNode.maxSize :434 -> DataDeduplicator.maxSize */
    int32_t device;          /* HIP device ordinal */
    int64_t max_block_bytes; /* largest block (dfs.blocksize, 128 MiB) */
    int32_t max_batch_blocks;/* <= 64 blocks per hdrf_reduce_batch call */
    int32_t index_log2;      /* index table capacity = 2^index_log2 entries (64 B each) */
    int64_t arena_slots;     /* container arena slots of container_max bytes each */
    int32_t segment_bytes;   /* chunking speculation segment (default 1 MiB) */
    int32_t keep_recipes;    /* keep recipes (SET blockId -> size|digests) on the host */
    int32_t timing;          /* record per-stage HIP events */
    int32_t debug_tag_bits;  /* test hook (SHA-1 only): keep only this many index-tag bits to force
                                tag collisions through the exact slow path; 0 = full 64-bit tag */
    int32_t n_ranks;         /* GPUs sharing ONE node-global index (1 = this GPU is the whole node) */
    int32_t rank;            /* this GPU's rank in [0, n_ranks) = index partition it owns */
    int32_t retain_containers; /* 1: durable containers (a DataNode): a closed container keeps its arena
                                  slot until hdrf_drain_containers has handed it out, and a submit that
                                  could need such a slot returns HDRF_E_CAPACITY; 0 (default): the
                                  arena is a ring cache of the newest containers (benchmarks, tests) */
} hdrf_cfg;

/* Per-block result of hdrf_reduce_block (caller-owned host arrays; NULL to skip). */
typedef struct {
    int64_t n_chunks;        /* out */
    int64_t store_size;      /* out: bytes of new chunks (DataDeduplicator.storeSize :91,355) */
    int64_t capacity;        /* in: entries available in the arrays below */
    uint32_t *offsets;       /* chunk END offsets (DataDeduplicator.chunking :264-307) */
    uint8_t *digests;        /* n * H bytes (threadedHasher :578-641) */
    uint8_t *is_new;         /* chunkMeta.newChunk (DN/chunkMeta.java:35-60) */
    uint32_t *container_id;  /* new chunks: chunkMeta.blockID (:799) */
    uint32_t *container_pos; /* new chunks: chunkMeta.blockStart (:800) */
} hdrf_block_result;

int hdrf_default_cfg(hdrf_cfg *cfg);
/* DataNode.initializeDD (DN/DataNode.java:486-534) + JedisPool("localhost") (DN/DataDeduplicator.java:119) */
int hdrf_open(const hdrf_cfg *cfg, hdrf_ctx **out);
int hdrf_close(hdrf_ctx *ctx);
const char *hdrf_last_error(const hdrf_ctx *ctx);
int hdrf_digest_len(const hdrf_ctx *ctx);              /* DataNode.hash_length (:528-532) */

/* Write path, one block from host memory: replaces `new DataDeduplicator(bf1, blockId)`
 * launched by DDRunner (DN/DDRunner.java:26-36, DN/BlockReceiver.java:1258-1261).
 * Copies H2D, reduces, updates the index / containers / recipe / allocator. */
int hdrf_reduce_block(hdrf_ctx *ctx, uint64_t block_id, const uint8_t *data, uint64_t len,
                      hdrf_block_result *out);

/* Write path, a batch of device-resident blocks in arrival order (the FIFO order of
 * DN/DataDeduplicator.java:124-158).  data[i] must stay valid until the call returns and
 * provide readable[i] >= len[i] + 64 bytes.  Results of the batch stay on the device until
 * the next reduce call and are read with hdrf_batch_*. */
int hdrf_reduce_batch(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                      const uint64_t *readable, const uint64_t *block_ids);

/* Pipelined form of hdrf_reduce_batch: hdrf_submit_batch enqueues the batch (chunking, SHA and
 * index + store on three HIP streams, in block order; under compressor 2 the batch's LZ4 pass runs
 * on one of two LZ4 streams, so consecutive batches' passes overlap) and returns; hdrf_wait_batch
 * completes the
 * OLDEST submitted batch and makes it the one hdrf_batch_* report.  At most HDRF_PIPELINE_DEPTH
 * batches are in flight: a submit beyond that returns HDRF_E_CAPACITY (call hdrf_wait_batch
 * first), so every submit pairs with exactly one wait.  The device buffers of a batch must stay
 * valid until it is completed.  Chunking of batch k+1 overlaps hashing of batch k and the
 * index/store stage of batch k-1 (latency-bound walk, VALU-bound SHA, HBM-bound store); the
 * bench keeps three batches in flight (five under compressor 2, where a batch's LZ4 pass outlasts
 * the front halves of the next ones).  Views (index, containers, allocator) complete all batches
 * first. */
#define HDRF_PIPELINE_DEPTH 5
int hdrf_submit_batch(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                      const uint64_t *readable, const uint64_t *block_ids);
int hdrf_wait_batch(hdrf_ctx *ctx);
/* The streaming DataNode write path (BASELINE config 5; the hook's bf1 handed over at
 * DN/BlockReceiver.java:1258-1261): host-resident blocks are copied H2D on a side stream
 * (hipMemcpyAsync from pinned memory overlaps the kernels of the batches in flight) into the
 * batch slot's staging buffer, then reduced exactly as hdrf_submit_batch.  The host buffers must
 * stay valid and unmodified until the batch completes (hdrf_wait_batch).  No 16-B alignment or
 * slack is required of host buffers. */
int hdrf_submit_host(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *host_data, const uint64_t *len,
                     const uint64_t *block_ids);
/* Packet-granular receive (DN/BlockReceiver.java:877-896, 1258-1261): hdrf_rx_begin reserves one of
 * 16 device receive buffers for a block (blocks received concurrently, as a DataNode runs one
 * DataXceiver per block being written); hdrf_append_packet copies each packet as it arrives into the
 * buffer's own pair of pinned 4 MiB staging chunks (the packet may be reused when the call returns)
 * and sends every full chunk H2D on a side stream, overlapped with the next packets and with the
 * blocks in flight.  The packets of one receive buffer come from one thread at a time (the block's
 * receiver); hdrf_append_packet does not take the context lock, so receivers of different blocks
 * copy concurrently;
 * hdrf_submit_slot submits the received block as a one-block batch with no copy left (pair it
 * with hdrf_wait_batch like hdrf_submit_batch; HDRF_E_CAPACITY when the pipeline is full).  The
 * buffer is free again when that batch completes; hdrf_rx_begin returns HDRF_E_CAPACITY while all
 * sixteen are in use.  hdrf_rx_cancel gives back a buffer whose block is abandoned (the client was
 * lost mid-block; the reference drops bf1): its receiver must have stopped appending.  A packet
 * that would take the block past max_block_bytes is refused (HDRF_E_INVAL) and copies nothing.
 * hdrf_reset refuses (HDRF_E_INVAL) while a buffer is receiving; hdrf_close requires every
 * receiver to have stopped.  hdrf_submit_slots submits n <= max_batch_blocks received blocks
 * (receive buffers listed in arrival order) as ONE batch: a DataNode whose receivers finished several
 * blocks since its last submit hands them over together (the FIFO order is the list order), so the
 * per-batch index / store passes are shared; the buffers are free again when that batch completes. */
int hdrf_rx_begin(hdrf_ctx *ctx, uint64_t block_id, int32_t *rx);
int hdrf_append_packet(hdrf_ctx *ctx, int32_t rx, const uint8_t *data, uint64_t len);
int hdrf_submit_slot(hdrf_ctx *ctx, int32_t rx);
int hdrf_submit_slots(hdrf_ctx *ctx, int32_t n, const int32_t *rx);
int hdrf_rx_cancel(hdrf_ctx *ctx, int32_t rx);
/* Stream-mode schemes (DataNode.compressor 0/3/4/5: the whole block through a Hadoop codec,
 * DN/BlockReceiver.java:822-894,1238-1256).  codec 4 = Lz4Codec, 0 = SnappyCodec, 3 = LzopCodec
 * (hadoop-lzo: LZO1X-1 blocks in an lzop file; the header's mtime is hdrf_set_lzop_mtime's value,
 * default 0, where the reference writes the wall clock), 5 = GzipCodec: the file
 * the reference writes to chunkDir+id when the block arrives as write()s of the given sizes (one
 * per packet, summing to len) followed by close().  dev_data needs len + 64 readable bytes.
 * Returns the file length (written to out), HDRF_E_CAPACITY if cap is too small,
 * HDRF_E_UNSUPPORTED for other codecs.  Codec 5's file does not depend on the write sizes
 * (zlib level 6 fed through Hadoop's ZlibCompressor); they must still add up to len.
 * Records the block length (SET id -> BE32(len)) for hdrf_block_length. */
int64_t hdrf_stream_block(hdrf_ctx *ctx, int32_t codec, uint64_t block_id, const uint8_t *dev_data, uint64_t len,
                          uint64_t readable, const uint64_t *writes, int32_t nwrites, uint8_t *out, int64_t cap);
/* hdrf_stream_block for a host-resident block (copied H2D first; no alignment or slack needed). */
int64_t hdrf_stream_block_host(hdrf_ctx *ctx, int32_t codec, uint64_t block_id, const uint8_t *data, uint64_t len,
                               const uint64_t *writes, int32_t nwrites, uint8_t *out, int64_t cap);
/* Read side for container / block FILES (DataConstructor's Lz4Codec input stream,
 * DN/DataConstructor.java:171-176,495-500): hdrf_lz4_file_decode decodes a Hadoop Lz4Codec file
 * (BlockCompressorStream framing, as written by compressor 2 containers and compressor 4 blocks)
 * on the GPU into dev_out; returns the raw length (HDRF_E_INVAL on a malformed file).
 * hdrf_container_load makes container `id` readable for hdrf_reconstruct* again from its chunkDir
 * file (lz4 = 1 for a closed container's Lz4Codec file, 0 for raw bytes) after its arena slot was
 * reused or the DataNode restarted; hdrf_container_unload frees that copy. */
int64_t hdrf_lz4_file_decode(hdrf_ctx *ctx, const uint8_t *file, int64_t flen, uint8_t *dev_out, int64_t cap);
/* The same for a stream-mode block file of codec 0 (SnappyCodec), 3 (LzopCodec: lzop header and
 * its checksum checked, LZO1X blocks decoded on the GPU), 4 (Lz4Codec) or 5 (GzipCodec:
 * gzip members, inflated on the GPU, CRC-32 and ISIZE checked): the compression-only decoders of
 * DataConstructor (DN/DataConstructor.java:102-220).  HDRF_E_INVAL on a malformed file. */
int64_t hdrf_stream_file_decode(hdrf_ctx *ctx, int32_t codec, const uint8_t *file, int64_t flen, uint8_t *dev_out,
                                int64_t cap);
/* The mtime field of the lzop headers hdrf_stream_block writes for codec 3 (LzopOutputStream puts
 * System.currentTimeMillis() / 1000 there, the only bytes of the file that are not a function of
 * the block). */
int hdrf_set_lzop_mtime(hdrf_ctx *ctx, uint32_t mtime);
/* Stage 1 of the GPU compressor 5 (GzipCodec = zlib level 6 deflate_slow, DN/BlockReceiver.java:
 * 858-873): for every position p of the len device bytes, the answer zlib's
 * longest_match gives at p with a 128-candidate chain (out128, prev_length < 8) and a 32-candidate
 * chain (out32, prev_length 8..15): (len << 16) | distance, 0 when no match of >= 3 bytes, bit 31
 * when the head candidate is a window-base position at distance exactly MAX_DIST.  dev_prev is
 * len u32 of scratch (the hash-chain predecessor + 1).  Synchronous on the context's stream. */
int hdrf_gzip_match_pass(hdrf_ctx *ctx, const uint8_t *dev_data, uint64_t len, uint32_t *dev_prev,
                         uint32_t *dev_out128, uint32_t *dev_out32);
/* Stage 2 of the GPU compressor 5: zlib's lazy parse (deflate_slow) over stage 1's answers.
 * dev_syms (len + 1 u32) receives (dist << 8) | lc per symbol (dist 0: literal lc; else lc =
 * length - 3); dev_blks (5 * (len / 16383 + 2) int64) one row per deflate block (symbol end,
 * block_start, strstart, window base, last); dev_cnt (2 int64) = {symbols, blocks}. */
int hdrf_gzip_parse(hdrf_ctx *ctx, const uint8_t *dev_data, uint64_t len, const uint32_t *dev_m128,
                    const uint32_t *dev_m32, uint32_t *dev_syms, int64_t *dev_blks, int64_t *dev_cnt);
int hdrf_container_load(hdrf_ctx *ctx, uint32_t id, const uint8_t *file, int64_t flen, int32_t lz4);
int hdrf_container_unload(hdrf_ctx *ctx, uint32_t id);
/* Restore a DataNode from its persisted state (the Redis keys + chunkDir files), on a fresh or
 * reset context: hdrf_index_load SETs digest -> 11-B value for n rows (keys n*H bytes, vals n*11,
 * e.g. the output of hdrf_index_dump); hdrf_allocator_load SETs "blockID" (24 B, as returned by
 * hdrf_allocator) and reopens each storer range's open container from its file (open_len[t] < 0:
 * no file); hdrf_recipe_load SETs longToBytes(id,4) -> recipe.  Blocks reduced afterwards, and
 * their containers, are those of a DataNode that never stopped. */
int hdrf_index_load(hdrf_ctx *ctx, const uint8_t *keys, const uint8_t *vals, int64_t n);
int hdrf_allocator_load(hdrf_ctx *ctx, const uint8_t alloc24[24], const uint8_t *const *open_files,
                        const int64_t *open_len);
int hdrf_recipe_load(hdrf_ctx *ctx, uint64_t block_id, const uint8_t *recipe, int64_t len);
/* Pinned (page-locked) host memory for hdrf_submit_host buffers. */
int hdrf_host_alloc(hdrf_ctx *ctx, uint64_t bytes, void **out);
int hdrf_host_free(hdrf_ctx *ctx, void *p);
/* Number of blocks of the batch hdrf_batch_* report (the last completed one). */
int hdrf_batch_nblocks(hdrf_ctx *ctx);

int hdrf_batch_info(hdrf_ctx *ctx, int32_t b, int64_t *n_chunks, int64_t *store_size);
int hdrf_batch_offsets(hdrf_ctx *ctx, int32_t b, uint32_t *out, int64_t cap);
int hdrf_batch_digests(hdrf_ctx *ctx, int32_t b, uint8_t *out, int64_t cap_bytes);
int hdrf_batch_is_new(hdrf_ctx *ctx, int32_t b, uint8_t *out, int64_t cap);
int hdrf_batch_placement(hdrf_ctx *ctx, int32_t b, uint32_t *cid, uint32_t *pos, int64_t cap);

/* Index (Redis) views. GET digest -> 11-byte chunkMeta value (DN/chunkMeta.java:62-77).
 * Returns 1 if found, 0 if absent, <0 on error. */
int hdrf_index_get(hdrf_ctx *ctx, const uint8_t *digest, uint8_t out11[11]);
int64_t hdrf_index_count(hdrf_ctx *ctx);
/* Probe lengths of the last completed batch: each chunk's distance (entries) from its home slot to
 * the entry its digest resolved to (linear probing); sum, max and chunk count.  Measurement only. */
int hdrf_probe_stats(hdrf_ctx *ctx, int64_t *probe_sum, int64_t *probe_max, int64_t *chunks);
/* All (digest, value) pairs sorted by digest; returns count (or HDRF_E_CAPACITY). */
int64_t hdrf_index_dump(hdrf_ctx *ctx, uint8_t *keys, uint8_t *vals, int64_t cap);
/* GET "blockID": 24-byte allocator (utilities.blockIDtoBytes, DN/utilities.java:66-75).
 * Returns 1 if the key exists (a block was reduced), 0 otherwise. */
int hdrf_allocator(hdrf_ctx *ctx, uint8_t out24[24]);
/* GET longToBytes(blockId,4): recipe [BE32 size | digests] (DataDeduplicator.storeDB :372-392).
 * Returns length, 0 if absent; HDRF_E_CAPACITY if cap is too small (needs keep_recipes). */
int64_t hdrf_recipe_get(hdrf_ctx *ctx, uint64_t block_id, uint8_t *out, int64_t cap);
/* FsDatasetImpl.getLength for 0-byte replicas (DN/fsdataset/impl/FsDatasetImpl.java:736-763). */
int64_t hdrf_block_length(hdrf_ctx *ctx, uint64_t block_id);
/* Container file chunkDir+id as it is now (the batches in flight complete first).  Returns length;
 * *closed = 1 once it overflowed.  Raw bytes, except closed containers under compressor 2: the
 * Lz4Codec file the storer rewrote (:770-779).  HDRF_E_NOTFOUND if it never existed or its arena
 * slot was recycled (cfg.retain_containers = 0), or after a drain handed it out and its slot was
 * reused (retain_containers = 1: the file is the caller's then). */
int64_t hdrf_container_read(hdrf_ctx *ctx, uint32_t id, uint8_t *out, int64_t cap, int32_t *closed);

/* Durable containers (cfg.retain_containers = 1): what the storers wrote to chunkDir since the
 * last drain (DN/DataDeduplicator.java:748-818).  Each event is one file operation:
 *   closed = 1   the container closed (:748-786): write nbytes bytes at file_off of chunkDir+id and
 *                the file is final.  Under compressor 2 file_off = 0 and the bytes are the whole
 *                Lz4Codec file (rewrite it).  Under compressor 1 the storer's rewrite (prevData ||
 *                buffer) leaves the bytes already handed out in place, so only the rest travels:
 *                file_off = the file's length so far (0 when nothing was handed out yet)
 *   closed = 0   the open container grew: write nbytes bytes at file_off (= the file's length so
 *                far) of chunkDir+id, creating it when file_off == 0 (:806-818)
 * The bytes of event i are out[data_off, data_off + nbytes).  Events come in order (closes in
 * close order, then the open containers) and whole; returns the number written, 0 when nothing is
 * pending, HDRF_E_CAPACITY (and *need = the next event's bytes) when not even one fits.  Call again
 * until it returns 0.  Hands out what the COMPLETED batches (hdrf_wait_batch) produced; batches
 * still in flight keep running (their containers come with a later drain), so a DataNode drains
 * after every hdrf_wait_batch without stalling the pipeline.  The copies run on a stream of their
 * own, beside the H2D copies of later blocks.  A drained closed container's slot may then be
 * reused; read it back with hdrf_container_load. */
typedef struct {
    uint32_t id;             /* container id (utilities.bytesToBlockID ranges, DN/utilities.java:36-75) */
    int32_t closed;
    int64_t file_off;
    int64_t nbytes;
    int64_t data_off;
} hdrf_container_event;
int64_t hdrf_drain_containers(hdrf_ctx *ctx, hdrf_container_event *ev, int64_t ev_cap, uint8_t *out, int64_t out_cap,
                              int64_t *need);

/* Arrival tickets (AIWriteQueue, DN/DataDeduplicator.java:124-158): take one when a block arrives
 * (BlockReceiver, before its DDRunner starts), reduce with it from any thread: a ticketed call waits
 * until every earlier ticket has been reduced or cancelled, so the index / containers / recipes
 * are those of the arrival order.  A ticket that will never be used must be cancelled. */
int hdrf_ticket_take(hdrf_ctx *ctx, uint64_t *ticket);
int hdrf_ticket_cancel(hdrf_ctx *ctx, uint64_t ticket);
int hdrf_reduce_block_ticketed(hdrf_ctx *ctx, uint64_t ticket, uint64_t block_id, const uint8_t *data, uint64_t len,
                               hdrf_block_result *out);

/* Read side: DataConstructor(blkID, recipe).data (DN/DataConstructor.java:73-250, 360-531), the
 * rebuild BlockSender serves on READ_BLOCK (DN/BlockSender.java:612-619).  Every recipe digest
 * is looked up in the index; its chunk, container[start, stop), lands at the running sum of the
 * chunk lengths.  hdrf_reconstruct writes to device memory and returns the block size;
 * hdrf_reconstruct_block uses the context's stored recipe and copies to host memory.  The
 * containers must still be resident (HDRF_E_NOTFOUND otherwise).  Single-node contexts. */
int64_t hdrf_reconstruct(hdrf_ctx *ctx, const uint8_t *recipe, int64_t recipe_len, uint8_t *dev_out, int64_t cap);
int64_t hdrf_reconstruct_block(hdrf_ctx *ctx, uint64_t block_id, uint8_t *out, int64_t cap);

/* The same read on a node-global context (cfg.n_ranks = G > 1): the node's ONE index is
 * partitioned over the ranks, and a container's bytes are spread over the ranks that placed
 * chunks into it, so every rank takes part (hdrf_amd/node.py NodeRank.reconstruct_block; the
 * shared Redis of DN/DataConstructor.java:360-417 serves any DataNode):
 *   1. every rank gets the block's n recipe digests (n * digest_len bytes, host);
 *      hdrf_gx_read_locate fills loc[4k..4k+3] = {container id, start, stop, placing rank + 1}
 *      for the digests it owns (first digest word mod G == rank) and zeros for the others;
 *      returns how many it owns, HDRF_E_NOTFOUND if an owned digest is absent;
 *   2. the G loc arrays are summed (the rows are disjoint);
 *   3. hdrf_gx_read_fill writes, at each chunk's block offset (running sum of stop - start) of
 *      dev_out (zeroed by the caller), the chunks this rank placed; returns the bytes written
 *      (HDRF_E_NOTFOUND when such a chunk's container left the arena ring);
 *   4. the G partial blocks summed byte-wise (disjoint) on the reading rank are the block; the
 *      returned counts sum to the recipe size.
 * Call between batches (no hdrf_gx_* batch in flight); both first complete the last batch's commit
 * and arena copy on this rank (as hdrf_gx_sync, whose commit error they report). */
int64_t hdrf_gx_read_locate(hdrf_ctx *ctx, const uint8_t *digests, int64_t n, uint32_t *loc);
int64_t hdrf_gx_read_fill(hdrf_ctx *ctx, const uint32_t *loc, int64_t n, uint8_t *dev_out, int64_t cap);

/* Device memory helpers for callers without their own allocator (bench, tests). */
int hdrf_dev_alloc(hdrf_ctx *ctx, uint64_t bytes, void **out);
int hdrf_dev_free(hdrf_ctx *ctx, void *p);
int hdrf_memcpy_h2d(hdrf_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int hdrf_memcpy_d2h(hdrf_ctx *ctx, void *dst, const void *src, uint64_t bytes);
int hdrf_synchronize(hdrf_ctx *ctx);

/* Synthetic corpus generator (BASELINE config 2; spec in DESIGN.md §Corpus):
 * block b, segment s = splitmix64 words keyed by roots[b*segs_per_block+s]. */
int hdrf_corpus_fill(hdrf_ctx *ctx, uint8_t *dev, const uint32_t *roots_host, int64_t nblocks,
                     int64_t segs_per_block, int64_t seg_bytes, uint64_t seed);
/* Same with mixed != 0: BASELINE config 4's mixed-entropy segments (random / text / binary). */
int hdrf_corpus_fill_kind(hdrf_ctx *ctx, uint8_t *dev, const uint32_t *roots_host, int64_t nblocks,
                          int64_t segs_per_block, int64_t seg_bytes, uint64_t seed, int32_t mixed);

/* Per-stage device time (ms) accumulated since the last reset, measured with HIP events on
 * the streams the stages run on (cfg.timing = 1): [0] lane_walk_kernel, [1] stitch (repair / path /
 * count / scan / copy / fallback), [2] sha_full_kernel, [3] sha_tail_kernel, [4] idx_claim_kernel,
 * [5] idx_apply_kernel, [6] idx_slow+decide, [7] new-byte scans, [8] flush_kernel, [9] place_kernel,
 * [10] lz4 (compressor 2), [11] gmax_kernel (granule maxima); node-global contexts also
 * [12] local aggregation + X1 records, [13] owner claim..finish, [14] gx_decide, [15] flush function,
 * [16] device allocator scan, [17] placement (part 1), [18] commit, and the gaps on the back stream
 * that the caller's exchanges fill: [19] X1 (+ the host), [20] X2, [21] descriptor all-gather,
 * [22] X3 (+ the host); [7] / [8] / [9] are the scans, the flush walk and the arena copy. */
int hdrf_stage_times(hdrf_ctx *ctx, double *ms, int32_t n, int32_t reset);
/* Reduction totals since the last reset (this context's blocks): the dedup / compression ratio
 * of the node is logical_bytes / (closed_file_bytes + open_bytes [+ recipe_bytes]). */
typedef struct {
    int64_t blocks, chunks;
    int64_t logical_bytes;       /* bytes of the reduced blocks */
    int64_t new_bytes;           /* sum of storeSize (DataDeduplicator.storeSize :355) */
    int64_t closed_containers;
    int64_t closed_raw_bytes;    /* container bytes of closed containers */
    int64_t closed_file_bytes;   /* their file sizes (Lz4Codec stream under compressor 2) */
    int64_t open_bytes;          /* raw bytes of the open containers (lastBlockID[0..2]) */
    int64_t recipe_bytes;        /* recipes: BE32 size + digests (storeDB :372-392) */
} hdrf_stats;
int hdrf_get_stats(hdrf_ctx *ctx, hdrf_stats *out);

/* Reset the index, containers, allocator and recipes (a fresh DataNode + Redis); completes
 * the batches in flight first.  HDRF_E_INVAL while a packet receive is open (hdrf_rx_begin not
 * yet followed by hdrf_submit_slot or hdrf_rx_cancel). */
int hdrf_reset(hdrf_ctx *ctx);
/* The same without completing the batches in flight: they complete against the old state, and the
 * next submit (node-global contexts: the next hdrf_gx_front_launch, every rank alike) starts the fresh
 * DataNode, so its front half overlaps the old batches' back halves.  Node-global contexts make the
 * switch in that batch's hdrf_gx_owner (the old batches' owner phases, enqueued after this call, still
 * use the old index epoch) and reset the host side in its hdrf_gx_place_wait.  Views and restores (hdrf_index_*, hdrf_*_load, reconstruct, container
 * reads, hdrf_synchronize) complete every batch first, as always, and a reset still pending then (no
 * submit since) is applied before they run, so they see the fresh DataNode and a restore is kept.
 * cfg.retain_containers: drain the old batches' containers as they complete (hdrf_wait_batch,
 * hdrf_drain_containers); while any old container (closed, or bytes of an open one) is not handed
 * out, hdrf_wait_batch on the fresh DataNode's first batch fails with HDRF_E_INVAL and leaves that
 * batch in flight (drain, then wait again), and the views above fail with HDRF_E_INVAL (a view that
 * must complete the batch anyway drops those containers and marks the context for hdrf_reset,
 * HDRF_E_CAPACITY). */
int hdrf_reset_async(hdrf_ctx *ctx);

/* ---- Node-global index over n_ranks GPUs (BASELINE config 3) -------------------
 * All DataNodes of one host share one Redis (JedisPool("localhost"), DN/DataDeduplicator.java:119),
 * one "blockID" allocator (:165-172,:389), one chunkDir and one FIFO (:124-158): the node is ONE
 * reduction over the global block sequence.  With n_ranks > 1 each context owns the index
 * partition {digest : first digest word mod n_ranks == rank} and reduces the blocks it receives;
 * a global batch is rank-major (rank r's blocks take batch positions [gbase_r, gbase_r + nblocks_r)).
 * The caller moves the records between ranks (all-to-all over RCCL/xGMI, hdrf_amd/node.py).
 * Buffers are device pointers laid out [n_ranks][cap][words] (region d = peer d); counts are
 * host int64[n_ranks].  Per global batch, every rank calls, in order:
 *   hdrf_gx_front  -> X1 send (records for each owner)      all-to-all X1
 *   hdrf_gx_owner  <- X1 recv, -> X2 send (responses)        all-to-all X2 (reverse counts)
 *   hdrf_gx_decide <- X2 recv
 *   hdrf_gx_flush_fn -> this rank's flush descriptor             all-gather of the descriptors
 *   hdrf_gx_alloc_scan <- every rank's descriptor: its allocator in + the node's after the batch
 *                     (or the device forms: hdrf_gx_flush_fn_dev / hdrf_gx_alloc_scan_dev)
 *   hdrf_gx_flush  <- alloc_in (from the scan; or, without the scan, rank r gets rank r-1's
 *                     state over a rank-to-rank chain, rank 0 the node's)
 *   hdrf_gx_place  -> X3 send (locations of new entries)     all-to-all X3 (receive counts from
 *                     hdrf_gx_x3_counts: no count exchange)
 *   hdrf_gx_commit <- X3 recv
 * hdrf_reduce_block / hdrf_reduce_batch return HDRF_E_INVAL on such a context. */
#define HDRF_ALLOC_STATE_BYTES 128
typedef struct {
    int64_t cap;             /* records per peer region (all three exchanges) */
    int32_t x1_words;        /* u32 words per X1 record (digest words + batch position + count) */
    int32_t x2_words;        /* 2: owner slot, flags */
    int32_t x3_words;        /* 4: owner slot, container id, start, stop */
    int32_t depth;           /* node-global batches in flight (fronts launched ahead, HDRF_GX_DEPTH) */
    int64_t fn_bytes;        /* bytes of one rank's packed flush descriptor (hdrf_gx_flush_fn_dev) */
} hdrf_gx_layout;
int hdrf_gx_layout_get(hdrf_ctx *ctx, hdrf_gx_layout *out);
int hdrf_gx_front(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                  const uint64_t *readable, const uint64_t *block_ids, uint32_t gbase, uint32_t *x1_send,
                  int64_t *send_counts);
/* hdrf_gx_front split in two: launch the front halves of the next batches (chunking on one stream,
 * SHA on a second, the local aggregation and X1 records on a third, each batch in its own slot)
 * before running the oldest batch's owner .. commit phases (the back stream), then wait for the
 * oldest launched front's X1 send counts.  At most hdrf_gx_layout.depth batches are in the
 * node-global pipeline (launched and not committed); fronts are waited and backs run in launch
 * order.  A slot is reused only after its previous batch's back phases finished on the device. */
int hdrf_gx_front_launch(hdrf_ctx *ctx, int32_t nblocks, const uint8_t *const *dev_data, const uint64_t *len,
                         const uint64_t *readable, const uint64_t *block_ids, uint32_t gbase, uint32_t *x1_send);
int hdrf_gx_front_wait(hdrf_ctx *ctx, int64_t *send_counts);
int hdrf_gx_owner(hdrf_ctx *ctx, const uint32_t *x1_recv, const int64_t *recv_counts, uint32_t *x2_send);
int hdrf_gx_decide(hdrf_ctx *ctx, const uint32_t *x2_recv);
/* The container allocator of a node-global batch without a rank-to-rank chain.  Each storer
 * range's flush walk (DN/DataDeduplicator.java:702-818: close when curPos + len > maxSize) depends
 * on the allocator a rank receives only through the open container's fill; hdrf_gx_flush_fn
 * (after hdrf_gx_decide) tabulates that function on the GPU into desc (int64 words; returns the
 * count, or -(count + 1000) when cap is too small).  With every rank's descriptor (rank order,
 * concatenated, lens[n_ranks]) hdrf_gx_alloc_scan computes this rank's incoming allocator
 * (alloc_in, the exclusive scan from the state after the previous batch) and the node's state
 * after the batch (alloc_final); hdrf_gx_place verifies the prediction against the flush walk. */
int64_t hdrf_gx_flush_fn(hdrf_ctx *ctx, int64_t *desc, int64_t cap);
int hdrf_gx_alloc_scan(hdrf_ctx *ctx, const int64_t *descs, const int64_t *lens, uint8_t *alloc_in,
                       uint8_t *alloc_final);
/* alloc_in: HDRF_ALLOC_STATE_BYTES from the previous rank or the scan (NULL: this context's own
 * state); alloc_out receives the state after this rank's blocks (NULL after a scan: no host
 * round trip). */
int hdrf_gx_flush(hdrf_ctx *ctx, const uint8_t *alloc_in, uint8_t *alloc_out);
/* The allocator scan without host round trips (the back stream's order only): hdrf_gx_flush_fn_dev
 * (after hdrf_gx_decide) writes this rank's flush function as a fixed-size descriptor of
 * hdrf_gx_layout.fn_bytes into dev_desc; the caller all-gathers the G descriptors into dev_descs
 * (rank order, G x fn_bytes, e.g. an RCCL all-gather enqueued on hdrf_gx_stream); then
 * hdrf_gx_alloc_scan_dev composes them on the device from the node's allocator after the previous
 * batch, and hdrf_gx_flush(ctx, NULL, NULL) and hdrf_gx_place(ctx, NULL, ...) use the result
 * (hdrf_gx_place checks the flush walk against the scan's prediction). */
int hdrf_gx_flush_fn_dev(hdrf_ctx *ctx, void *dev_desc);
int hdrf_gx_alloc_scan_dev(hdrf_ctx *ctx, const void *dev_descs);
/* alloc_final: the node's state after the last rank's flush (becomes this context's state; NULL
 * after hdrf_gx_alloc_scan_dev, which computed it).  hdrf_gx_place = hdrf_gx_place_launch (placement,
 * X3 records and their read-back on the back stream, the arena copy on a stream of its own) +
 * hdrf_gx_place_wait (waits for the read-back: this rank's X3 send counts; the scan and the X3
 * counts are checked, the batch's hdrf_batch_* views become valid). */
int hdrf_gx_place(hdrf_ctx *ctx, const uint8_t *alloc_final, uint32_t *x3_send, int64_t *send_counts);
int hdrf_gx_place_launch(hdrf_ctx *ctx, const uint8_t *alloc_final, uint32_t *x3_send);
int hdrf_gx_place_wait(hdrf_ctx *ctx, int64_t *send_counts);
/* Node-global compressor 2 (between hdrf_gx_place and hdrf_gx_commit): every rank's allocator
 * state before and after its flush walk (hdrf_gx_alloc_io, 128 B each; all-gathered by the caller,
 * they tell every rank which rank holds which bytes of each container); the head pieces of a
 * container another rank closes are copied out of / into arena slots (hdrf_gx_piece: write = 0 reads
 * the bytes [off, off + n) of container id into dev and returns when they are there; write = 1
 * enqueues the copy from dev on the back stream and returns at once, so dev must stay valid until
 * hdrf_gx_compress has returned, which runs after the copies); then each rank compresses the
 * containers its flush walk closed (hdrf_gx_compress: the Lz4Codec files of DN/DataDeduplicator.java
 * :748-797, returns how many).  hdrf_amd/node.py plans and runs the transfers. */
int hdrf_gx_alloc_io(hdrf_ctx *ctx, uint8_t *alloc_in, uint8_t *alloc_out);
int hdrf_gx_piece(hdrf_ctx *ctx, uint32_t id, uint64_t off, uint64_t n, void *dev, int32_t write);
int hdrf_gx_compress(hdrf_ctx *ctx);
/* X3 receive counts (int64[n_ranks]) implied by this owner's hdrf_gx_owner decisions: one location
 * per entry created this batch, from the rank holding its minimum block.  Valid from hdrf_gx_place to
 * hdrf_gx_commit; hdrf_gx_commit refuses (HDRF_E_DEVICE) receive counts that differ from them. */
int hdrf_gx_x3_counts(hdrf_ctx *ctx, int64_t *recv_counts);
/* Enqueued on the back stream and not waited for: a device error it raises is reported by the next
 * hdrf_gx_place or by hdrf_gx_sync. */
int hdrf_gx_commit(hdrf_ctx *ctx, const uint32_t *x3_recv, const int64_t *recv_counts);
/* Complete every node-global batch in flight on this rank (all streams); reports a commit error. */
int hdrf_gx_sync(hdrf_ctx *ctx);
/* The stream the back phases (hdrf_gx_owner .. hdrf_gx_commit) run on (a hipStream_t).  A caller
 * that enqueues its X1 / X2 record exchanges on it (RCCL collectives issued on this stream,
 * torch.cuda.ExternalStream in hdrf_amd/node.py) needs no host synchronisation between an exchange
 * and the phase that reads its receive buffer: hdrf_gx_owner and hdrf_gx_decide only enqueue, and
 * a device error they raise is reported by hdrf_gx_place. */
int hdrf_gx_stream(hdrf_ctx *ctx, void **stream);

#ifdef __cplusplus
}
#endif
#endif
