"""ReductionScheme — the plugin API HDRF's README promises (README.md:3) and its DataNode hook
uses de facto:
  write: `new DataDeduplicator(ByteBuffer block, long blockId)` run by DDRunner
         (DN/DataDeduplicator.java:108, DN/DDRunner.java:20-36, DN/BlockReceiver.java:1258-1261)
  read:  `new DataConstructor(long blkID, byte[] recipe).data`   (DN/DataConstructor.java:46-73)
  length: FsDatasetImpl.getLength via Redis GET id               (DN/fsdataset/impl/FsDatasetImpl.java:736-763)

HipReductionScheme is the MI355X backend (libhdrf.so via ctypes; the Java DataNode binds the
same C-ABI through JNI).  Like DDRunner, `reduce` is one call per received
block in arrival order.
"""
import abc

from .lib import Context


class ReductionScheme(abc.ABC):
    """Abstract reduction scheme (one instance per DataNode)."""

    @abc.abstractmethod
    def reduce(self, block, block_id):
        """Reduce one received block (DataDeduplicator(ByteBuffer, long))."""

    @abc.abstractmethod
    def reconstruct(self, block_id):
        """Rebuild a block's bytes (DataConstructor(long, byte[]).data)."""

    @abc.abstractmethod
    def length(self, block_id):
        """Logical length of a reduced block (FsDatasetImpl.getLength for 0-byte replicas)."""


class HipReductionScheme(ReductionScheme):
    """GPU-backed scheme: `compressor` 1 (dedup) or 2 (dedup + Lz4Codec containers),
    DN/DataNode.java:438."""

    def __init__(self, hasher=0, device=0, compressor=1, **cfg):
        self.ctx = Context(hasher=hasher, compressor=compressor, device=device, **cfg)
        self.last = None

    def reduce(self, block, block_id):
        self.last = self.ctx.reduce_block(block, block_id)
        return self.last

    def reconstruct(self, block_id):
        return self.ctx.reconstruct_block(block_id).tobytes()

    def length(self, block_id):
        return self.ctx.block_length(block_id)

    def recipe(self, block_id):
        return self.ctx.recipe(block_id)

    def index_get(self, digest):
        return self.ctx.index_get(digest)

    def close(self):
        self.ctx.close()
