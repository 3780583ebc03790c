package org.apache.hadoop.hdfs.server.datanode;

import java.io.IOException;
import java.nio.ByteBuffer;

/**
 * The plugin API README.md:3 promises ("ReductionScheme abstract class ... enabled in
 * DataNode #438").  It mirrors the de-facto contract of the reference:
 *   reduce      = new DataDeduplicator(ByteBuffer block, long blockId)   (DataDeduplicator.java:108)
 *   reconstruct = new DataConstructor(long blkID, byte[] recipe).data    (DataConstructor.java:46-73)
 *   length      = FsDatasetImpl.getLength for 0-byte replicas            (FsDatasetImpl.java:736-763)
 */
public abstract class ReductionScheme implements AutoCloseable {
  /** Reduce one received block; {@code block.position()} is its length (DataDeduplicator.java:114). */
  public abstract void reduce(ByteBuffer block, long blockId) throws IOException;

  /** Rebuild the block bytes from the recipe stored under {@code blockId}. */
  public abstract byte[] reconstruct(long blockId) throws IOException;

  /** Logical length of a reduced block (recipe head). */
  public abstract long length(long blockId) throws IOException;

  @Override
  public void close() {}
}
