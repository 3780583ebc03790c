/*
 * hdrf_oracle.h — CPU restatement of HDRF's per-block reduction path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library, and only as the checker / CPU baseline.
 * The product path (hdrf_amd/, libhdrf.so) never links or calls it.
 *
 * Pinning status:
 *   - SHA-1 / SHA-224 digests: pinned to FIPS 180-4 known-answer vectors and to
 *     Python hashlib (the survey verified the reference's native hasher equals
 *     hashlib on 11 lengths).
 *   - chunk boundaries, dedup decisions, index values, containers, recipes,
 *     allocator: PARITY UNPINNED against the running reference (Java; no JDK,
 *     Redis or Hadoop jars exist here and the reference ships no tests for this
 *     path).  They are restated line by line from the cited Java sources and
 *     cross-checked against an independent pure-Python transliteration
 *     (oracle/pyref.py).
 */
#ifndef HDRF_ORACLE_H
#define HDRF_ORACLE_H
#include <stdint.h>
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

/* DataDeduplicator.chunking — DN/DataDeduplicator.java:264-307.
 * Writes the chunk END offsets (last detected boundary dropped, `size` appended)
 * into out[0..n); returns n, or -1 if out_cap is too small. */
int64_t hdrf_oracle_chunk(const uint8_t *data, int64_t size, uint32_t *out, int64_t out_cap);

/* FIPS 180-4 SHA-1 / SHA-224 (utilities.sha1hash/sha224hash, DN/utilities.java:98-137). */
void hdrf_oracle_sha1(const uint8_t *msg, uint64_t len, uint8_t out[20]);
void hdrf_oracle_sha224(const uint8_t *msg, uint64_t len, uint8_t out[28]);

/* Whole write path: DataDeduplicator(ByteBuffer, long) — DN/DataDeduplicator.java:108-217,
 * with Redis restated as an in-memory map and container files as in-memory byte vectors. */
typedef struct hdrf_oracle hdrf_oracle;
hdrf_oracle *hdrf_oracle_new(int hasher, int compressor, uint32_t max_size);
void hdrf_oracle_free(hdrf_oracle *o);
/* Store-size mode (call before the first block): the storers keep container LENGTHS, not bytes, and
 * no recipe is kept; chunks, digests, dedup decisions, index values, the allocator and storeSize are
 * unchanged (bench.py checks the whole corpus's storeSize with it, in a few GB of host memory).
 * hdrf_oracle_container / hdrf_oracle_recipe then report nothing. */
void hdrf_oracle_set_store_only(hdrf_oracle *o, int on);

/* Reduce one block.  Optional outputs (NULL to skip), each sized for cap chunks:
 *   offsets[n], digests[n*H], is_new[n], values[n*11] (the 11-byte value each chunk SETs).
 * Returns n (number of chunks) or a negative error. */
int64_t hdrf_oracle_reduce(hdrf_oracle *o, const uint8_t *data, int64_t size, int64_t block_id,
                           int64_t cap, uint32_t *offsets, uint8_t *digests, uint8_t *is_new,
                           uint8_t *values, int64_t *store_size);

/* GET digest -> 11-byte value; returns 1 if present. */
/* Threaded CPU baseline (bench.py cpu_baseline only): worker threads chunk + hash blocks ahead,
 * the ordered part handles them in arrival order; same results as hdrf_oracle_reduce in order. */
int64_t hdrf_oracle_reduce_many(hdrf_oracle *o, const uint8_t *const *blocks, const int64_t *sizes,
                                const int64_t *ids, int64_t nblocks, int nthreads, int64_t *store_sizes);
/* Per-block result buffers for hdrf_oracle_reduce_many_out (the arrays of hdrf_oracle_reduce). */
typedef struct {
    int64_t cap;
    uint32_t *offsets;
    uint8_t *digests, *is_new, *values;
} hdrf_oracle_out;
int64_t hdrf_oracle_reduce_many_out(hdrf_oracle *o, const uint8_t *const *blocks, const int64_t *sizes,
                                    const int64_t *ids, int64_t nblocks, int nthreads, int64_t *store_sizes,
                                    const hdrf_oracle_out *out, int64_t *counts);
/* The reference's concurrency shape, blocks serialised: per block 1 chunking thread + nhash hasher
 * threads over chunk ranges, then the ordered part (BASELINE.md CPU plan 1). */
int64_t hdrf_oracle_reduce_ref_shape(hdrf_oracle *o, const uint8_t *const *blocks, const int64_t *sizes,
                                     const int64_t *ids, int64_t nblocks, int nhash, int64_t *store_sizes);
int hdrf_oracle_index_get(const hdrf_oracle *o, const uint8_t *digest, uint8_t out11[11]);
int64_t hdrf_oracle_index_count(const hdrf_oracle *o);
/* Dump every (digest, value) pair, sorted by digest bytes. Returns count (or -needed if cap small). */
int64_t hdrf_oracle_index_dump(const hdrf_oracle *o, uint8_t *keys, uint8_t *vals, int64_t cap);
/* GET "blockID" -> 24 bytes; returns 1 if the key exists. */
int hdrf_oracle_allocator(const hdrf_oracle *o, uint8_t out24[24]);
/* GET longToBytes(blockId,4) -> recipe bytes; returns length, 0 if absent, -needed if cap small. */
int64_t hdrf_oracle_recipe(const hdrf_oracle *o, int64_t block_id, uint8_t *out, int64_t cap);
/* Container file chunkDir+id: returns length (-1 absent, -(needed+2) if cap too small).
 * *closed = 1 once the container was rewritten on overflow.  Raw bytes, except a closed
 * container under compressor 2, which is the Lz4Codec file (hdrf_oracle_hadoop_lz4_frame). */
int64_t hdrf_oracle_container(const hdrf_oracle *o, uint32_t id, uint8_t *out, int64_t cap, int *closed);

/* Compression stage (compressor == 2, DN/DataDeduplicator.java:770-779): lz4 r123 LZ4_compress
 * and Hadoop BlockCompressorStream framing (Lz4Codec, 256 KiB buffer).  Third-party, not in the
 * reference tree: compressed-byte parity vs Hadoop UNPINNED; see hdrf_oracle.c. */
int64_t hdrf_oracle_lz4_bound(int64_t n);
int64_t hdrf_oracle_lz4_compress(const uint8_t *src, int64_t n, uint8_t *dst);
int64_t hdrf_oracle_lz4_compress_modern(const uint8_t *src, int64_t n, uint8_t *dst, int rules);   /* tests: liblz4 >= 1.9 rules */
int64_t hdrf_oracle_lz4_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap);
int64_t hdrf_oracle_hadoop_lz4_bound(int64_t n);
int64_t hdrf_oracle_hadoop_lz4_frame(const uint8_t *src, int64_t n, uint8_t *dst);
int64_t hdrf_oracle_hadoop_lz4_unframe(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap);
/* Stream mode (compressor == 4, DN/BlockReceiver.java:846-855,887-894,1238-1256): the block goes
 * through Lz4Codec.createOutputStream(file) as one write() per received packet (sizes `writes`,
 * summing to the block length), then close().  Decodes with hdrf_oracle_hadoop_lz4_unframe. */
int64_t hdrf_oracle_hadoop_lz4_stream_bound(int64_t n, int64_t nwrites);
int64_t hdrf_oracle_hadoop_lz4_stream(const uint8_t *src, const int64_t *writes, int64_t nwrites, uint8_t *dst);

/* Stream mode compressor == 0 (Hadoop SnappyCodec, MAX_INPUT 218,422): snappy raw format
 * restated from google/snappy; pinned against pyarrow's bundled snappy, vs Hadoop UNPINNED. */
int64_t hdrf_oracle_snappy_bound(int64_t n);
int64_t hdrf_oracle_snappy_compress(const uint8_t *src, int64_t n, uint8_t *dst);
int64_t hdrf_oracle_snappy_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap);
/* Stream mode compressor == 5 (Hadoop GzipCodec over native zlib, level 6): zlib 1.2.11
 * deflate_slow + trees restated (hdrf_gzip.c); pinned byte for byte against this image's
 * zlib 1.2.11.  The file is one gzip member (header OS byte 3, CRC-32 + ISIZE trailer). */
int64_t hdrf_oracle_gzip_bound(int64_t n);
int64_t hdrf_oracle_gzip_compress(const uint8_t *src, int64_t n, uint8_t *dst);
/* the same, logging every longest_match call as (strstart, prev_length, length, match_start) */
int64_t hdrf_oracle_gzip_trace(const uint8_t *src, int64_t n, uint8_t *dst, int64_t *trace, int64_t tcap,
                               int64_t *ntrace);
/* the same, logging the parse: symbols ((dist << 8) | lc) and flushed blocks (5 int64 each) */
int64_t hdrf_oracle_gzip_symbols(const uint8_t *src, int64_t n, uint8_t *dst, uint32_t *syms, int64_t *nsyms,
                                 int64_t *blks, int64_t *nblks);
uint32_t hdrf_oracle_crc32(const uint8_t *p, int64_t n);
/* codec 0 (SnappyCodec) or 4 (Lz4Codec) stream file / its decoding */
int64_t hdrf_oracle_hadoop_stream_bound(int codec, int64_t n, int64_t nwrites);
int64_t hdrf_oracle_hadoop_stream(int codec, const uint8_t *src, const int64_t *writes, int64_t nwrites, uint8_t *dst);
int64_t hdrf_oracle_hadoop_unframe(int codec, const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap);

/* Synthetic corpus (shared spec with hdrf_amd corpus generator). */
uint64_t hdrf_oracle_mix64(uint64_t z);
void hdrf_oracle_corpus_roots(uint64_t seed, uint32_t dup_ppm, int64_t nblocks, int64_t segs_per_block,
                              uint32_t *roots);
void hdrf_oracle_corpus_fill(uint64_t seed, const uint32_t *roots, int64_t block, int64_t segs_per_block,
                             int64_t seg_bytes, uint8_t *out);

/* java.util.Random(seed).nextBytes in buffer_len pieces (DFSTestUtil.createFile,
 * hadoop-hdfs/src/test/java/org/apache/hadoop/hdfs/DFSTestUtil.java:441-450). */
void hdrf_oracle_java_random_bytes(int64_t seed, int32_t buffer_len, int64_t total, uint8_t *out);

#ifdef __cplusplus
}
#endif

/* LZOP stream mode (compressor 3): LZO1X-1 + hadoop-lzo LzopOutputStream framing (hdrf_lzo.c) */
int64_t hdrf_oracle_lzo1x_1_compress(const uint8_t *in, int64_t in_len, uint8_t *out);
int64_t hdrf_oracle_lzo1x_decompress(const uint8_t *in, int64_t in_len, uint8_t *out, int64_t cap);
int64_t hdrf_oracle_lzop_header(uint32_t mtime, uint8_t *dst);
int64_t hdrf_oracle_lzop_stream_bound(int64_t n, int64_t nwrites);
int64_t hdrf_oracle_lzop_stream(const uint8_t *src, const int64_t *writes, int64_t nwrites, uint32_t mtime,
                                uint8_t *dst);
int64_t hdrf_oracle_lzop_decode(const uint8_t *f, int64_t n, uint8_t *dst, int64_t cap);
#endif
