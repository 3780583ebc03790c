"""Per-kind LZ4 wave speed: a 64 MiB block of one corpus kind (config 4's random / text / binary
segments) through the stream-mode Lz4Codec path — 257 independent 261,100-B segments, one wave
each, so the kernel time is one wave's time for a whole segment of that kind."""
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from hdrf_amd.corpus import corpus_block_host, segment_kind  # noqa: E402
from hdrf_amd.lib import Context  # noqa: E402


def main():
    spb, seg = 64, 1 << 20
    ctx = Context(max_block_bytes=64 << 20, max_batch_blocks=1, index_log2=20, arena_slots=16)
    for kind, name in ((0, "random"), (1, "text"), (2, "binary")):
        roots = [r for r in range(1, 5000) if segment_kind(r) == kind][:spb]
        blk = corpus_block_host(7, np.array(roots, np.uint32), 0, spb, seg, mixed=True)
        ctx.stream_block_host(4, 1, blk, [blk.size])           # warm
        t = time.perf_counter()
        f = ctx.stream_block_host(4, 1, blk, [blk.size])
        dt = time.perf_counter() - t
        print(f"{name:7s} 64 MiB -> {len(f) / blk.size:.3f}x  {dt * 1e3:8.1f} ms wall  "
              f"{seg * spb / dt / 1e6 / 257:6.2f} MB/s per wave", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
