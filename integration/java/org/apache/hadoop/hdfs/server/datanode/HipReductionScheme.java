package org.apache.hadoop.hdfs.server.datanode;

import java.io.IOException;
import java.nio.ByteBuffer;

/**
 * MI355X backend: JNI over libhdrf.so (include/hdrf.h).  Selected where DataNode.compressor is
 * tested (DataNode.java:438, BlockReceiver.java:822-879) in place of `new DDRunner(bf1, id)`.
 * bf1 must be a direct ByteBuffer (BlockReceiver.java:877 allocates it with allocateDirect, or
 * allocPinned() for an overlapped H2D).
 *
 * Threads: every method may be called from any thread (the native context serialises calls).
 * Block order: reduce() reduces in call order; for the reference's FIFO (AIWriteQueue,
 * DataDeduplicator.java:124-158) take arrive() when the block is received and pass the ticket to
 * reduce(ticket, ...) from the block's own DDRunner-style thread.
 * Durability: containers are kept in HBM until drainContainers(chunkDir) has written them; call it
 * after every awaitOldest().  A reduction that could overwrite an undrained container fails with
 * IOException naming its recovery: "hdrf_drain_containers first" (drain, then retry) or, when the
 * blocks still in flight are what fills the ring, "hdrf_wait_batch, then hdrf_drain_containers"
 * (awaitOldest(), drainContainers(), then retry).
 */
public final class HipReductionScheme extends ReductionScheme {
  static { System.loadLibrary("hdrf_jni"); }   // libhdrf_jni.so -> libhdrf.so

  private long ctx;                            // hdrf_ctx*

  /** hasher: DataNode.hasher (0 SHA-1, 1 SHA-224); compressor: DataNode.compressor (1, 2). */
  public HipReductionScheme(int hasher, int compressor, int device, long maxBlockBytes) throws IOException {
    this(hasher, compressor, device, maxBlockBytes, 16);
  }

  /** maxBatchBlocks: most blocks one submitBlocks() hands over together (1..16). */
  public HipReductionScheme(int hasher, int compressor, int device, long maxBlockBytes, int maxBatchBlocks)
      throws IOException {
    ctx = open0(hasher, compressor, device, maxBlockBytes, maxBatchBlocks);
  }

  @Override
  public void reduce(ByteBuffer block, long blockId) throws IOException {
    if (!block.isDirect()) throw new IOException("HipReductionScheme needs a direct ByteBuffer");
    reduce0(ctx, block, block.position(), blockId);   // H2D copy happens before return
  }

  /** The block's place in the FIFO, taken when it is received (before its reducing thread starts). */
  public long arrive() throws IOException {
    return arrive0(ctx);
  }

  /** reduce() in arrival-ticket order: waits until every earlier ticket was reduced or cancelled. */
  public void reduce(long ticket, ByteBuffer block, long blockId) throws IOException {
    if (!block.isDirect()) { cancel0(ctx, ticket); throw new IOException("HipReductionScheme needs a direct ByteBuffer"); }
    reduceTicket0(ctx, ticket, block, block.position(), blockId);
  }

  /** A ticket whose block will not be reduced (the receive failed). */
  public void cancel(long ticket) throws IOException {
    cancel0(ctx, ticket);
  }

  /**
   * The storers' chunkDir writes since the last call (DataDeduplicator.java:748-818): closed
   * containers rewritten whole (Lz4Codec files under compressor 2), open containers appended.
   * Returns the number of file operations.
   */
  public int drainContainers(String chunkDir) throws IOException {
    return drain0(ctx, chunkDir);
  }

  /** Page-locked direct buffer for received blocks (reduceAsync copies it H2D on a side stream). */
  public ByteBuffer allocPinned(long bytes) throws IOException {
    return allocPinned0(ctx, bytes);
  }

  public void freePinned(ByteBuffer buf) throws IOException {
    freePinned0(ctx, buf);
  }

  /**
   * Streaming write path (BASELINE config 5): enqueue the received block and return at once; its
   * H2D copy runs on a side stream overlapped with the blocks already in flight.  `block` must
   * stay untouched until awaitOldest() has returned for it (keep a reference; BlockReceiver
   * allocates a fresh bf1 per block).  Completion is in submission order, like the FIFO
   * (DataDeduplicator.java:124-158).  At most HDRF_PIPELINE_DEPTH (5, include/hdrf.h) blocks are in
   * flight: a sixth reduceAsync throws IOException ("pipeline full") until awaitOldest() completed
   * one, so every reduceAsync pairs with exactly one awaitOldest.
   */
  public void reduceAsync(ByteBuffer block, long blockId) throws IOException {
    if (!block.isDirect()) throw new IOException("HipReductionScheme needs a direct ByteBuffer");
    submit0(ctx, block, block.position(), blockId);
  }

  /**
   * Packet-granular receive (BlockReceiver.java:877-896): begin a block, hand every packet over as
   * it arrives (copied before the call returns; its H2D overlaps the next packets and the blocks in
   * flight), then submit it.  Pair every submitBlock with one awaitOldest, like reduceAsync.
   */
  public int beginBlock(long blockId) throws IOException {
    return rxBegin0(ctx, blockId);
  }

  public void packet(int rx, ByteBuffer pkt, int off, int len) throws IOException {
    if (!pkt.isDirect()) throw new IOException("HipReductionScheme needs a direct ByteBuffer");
    if (off < 0 || len < 0 || off > pkt.capacity() - len)
      throw new IOException("packet range [" + off + ", +" + len + ") outside the buffer");
    packet0(ctx, rx, pkt, off, len);
  }

  public void submitBlock(int rx) throws IOException {
    submitSlot0(ctx, rx);
  }

  /**
   * Every block whose last packet arrived since the previous submit, handed over as ONE batch in
   * arrival order (the FIFO order is the array order): the blocks share one pass of the index and
   * store kernels.  One awaitOldest() completes the whole batch.
   */
  public void submitBlocks(int[] rx) throws IOException {
    submitSlots0(ctx, rx);
  }

  /**
   * Abandon a block being received (the client was lost mid-block; BlockReceiver drops bf1): the
   * receive buffer is free again.  Call it from BlockReceiver's error path, after the receiver
   * thread stopped calling packet().
   */
  public void abortBlock(int rx) throws IOException {
    rxCancel0(ctx, rx);
  }

  /** Complete the oldest block submitted with reduceAsync (its index/containers/recipe are final). */
  public void awaitOldest() throws IOException {
    wait0(ctx);
  }

  /**
   * Stream-mode schemes (DataNode.compressor 0 SnappyCodec, 3 LzopCodec, 4 Lz4Codec, 5 GzipCodec; BlockReceiver.java:
   * 826-873,887-894,1238-1256): the file the reference writes to chunkDir + blockId when the block
   * arrives as write()s of the given packet sizes followed by close().  The caller stores it and
   * the library records SET blockId -> BE32(length).
   */
  public byte[] streamBlock(int codec, ByteBuffer block, long blockId, long[] packetSizes) throws IOException {
    if (!block.isDirect()) throw new IOException("HipReductionScheme needs a direct ByteBuffer");
    return stream0(ctx, codec, block, block.position(), blockId, packetSizes);
  }

  /**
   * Stream-mode read (DataConstructor.java:102-220): the chunkDir + blockId file written by
   * streamBlock, decoded on the GPU through the codec (0 Snappy, 3 Lzop with its header checksum,
   * 4 Lz4, 5 Gzip with CRC-32/ISIZE checks); IOException on a malformed file or one whose length
   * differs from the recorded one.
   */
  public byte[] streamDecode(int codec, byte[] file, long blockId) throws IOException {
    return streamDecode0(ctx, codec, file, blockId);
  }

  @Override
  public byte[] reconstruct(long blockId) throws IOException {
    return reconstruct0(ctx, blockId);          // DataConstructor(blkID, recipe).data
  }

  @Override
  public long length(long blockId) throws IOException {
    return length0(ctx, blockId);
  }

  /** GET blockId -> recipe [BE32 size | digests] (storeDB, DataDeduplicator.java:372-392). */
  public byte[] recipe(long blockId) throws IOException {
    return recipe0(ctx, blockId);
  }

  @Override
  public void close() {
    if (ctx != 0) { close0(ctx); ctx = 0; }
  }

  private static native long open0(int hasher, int compressor, int device, long maxBlockBytes, int maxBatchBlocks)
      throws IOException;
  private static native byte[] reconstruct0(long ctx, long blockId) throws IOException;
  private static native void reduce0(long ctx, ByteBuffer direct, int len, long blockId) throws IOException;
  private static native void submit0(long ctx, ByteBuffer direct, int len, long blockId) throws IOException;
  private static native void wait0(long ctx) throws IOException;
  private static native long length0(long ctx, long blockId) throws IOException;
  private static native byte[] recipe0(long ctx, long blockId) throws IOException;
  private static native byte[] stream0(long ctx, int codec, ByteBuffer direct, int len, long blockId, long[] writes)
      throws IOException;
  private static native void close0(long ctx);
  private static native long arrive0(long ctx) throws IOException;
  private static native void reduceTicket0(long ctx, long ticket, ByteBuffer direct, int len, long blockId)
      throws IOException;
  private static native void cancel0(long ctx, long ticket) throws IOException;
  private static native int drain0(long ctx, String chunkDir) throws IOException;
  private static native ByteBuffer allocPinned0(long ctx, long bytes) throws IOException;
  private static native void freePinned0(long ctx, ByteBuffer buf) throws IOException;
  private static native int rxBegin0(long ctx, long blockId) throws IOException;
  private static native void packet0(long ctx, int rx, ByteBuffer pkt, int off, int len) throws IOException;
  private static native void submitSlot0(long ctx, int rx) throws IOException;
  private static native void submitSlots0(long ctx, int[] rx) throws IOException;
  private static native void rxCancel0(long ctx, int rx) throws IOException;
  private static native byte[] streamDecode0(long ctx, int codec, byte[] file, long blockId) throws IOException;
}
