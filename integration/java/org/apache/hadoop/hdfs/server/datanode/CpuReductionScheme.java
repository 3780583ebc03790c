package org.apache.hadoop.hdfs.server.datanode;

import java.io.IOException;
import java.nio.ByteBuffer;

import redis.clients.jedis.Jedis;

/**
 * The stock backend of ReductionScheme: the reference's own CPU path, unchanged, behind the
 * plugin API (SURVEY §8(b)).  A DataNode configured without a GPU keeps exactly today's behaviour:
 *   reduce      = new DDRunner(bf1, blockId).start()           (BlockReceiver.java:1261, DDRunner.java:26-36:
 *                 DataDeduplicator chunk/hash, the AIWriteQueue FIFO, Redis, the storers' chunkDir files)
 *   reconstruct = new DataConstructor(blockId, recipe).data    (BlockSender.java:572,615)
 *   length      = the recipe head, GET longToBytes(blockId, 4)  (FsDatasetImpl.java:736-763)
 */
public final class CpuReductionScheme extends ReductionScheme {

  @Override
  public void reduce(ByteBuffer block, long blockId) {
    new DDRunner(block, blockId).start();
  }

  @Override
  public byte[] reconstruct(long blockId) throws IOException {
    byte[] recipe = recipe(blockId);
    if (recipe == null) throw new IOException("no recipe for block " + blockId);
    return new DataConstructor(blockId, recipe).data;
  }

  @Override
  public long length(long blockId) {
    byte[] recipe = recipe(blockId);
    if (recipe == null) return 0;
    byte[] fsize = new byte[4];
    System.arraycopy(recipe, 0, fsize, 0, 4);
    return new utilities().bytesToLong(fsize, 4);
  }

  private static byte[] recipe(long blockId) {
    Jedis jedis = new Jedis("localhost");                  // DataDeduplicator.java:119 uses the same server
    try {
      return jedis.get(new utilities().longToBytes(blockId, 4));
    } finally {
      jedis.close();
    }
  }
}
