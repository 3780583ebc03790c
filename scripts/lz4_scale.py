"""LZ4 aggregate throughput vs segments in flight, per config-4 corpus kind: one device-resident
block of k x 64 MiB of a single kind through the stream-mode Lz4Codec path (one wave per
261,100-B piece).  Run under rocprofv3 --kernel-trace; the lz4_list_kernel durations are the
numbers (scripts/r02_lzs.sh)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hdrf_amd.corpus import segment_kind  # noqa: E402
from hdrf_amd.lib import Context  # noqa: E402


def main():
    seg = 1 << 20
    sizes = [int(x) for x in os.environ.get("LZS_MIB", "64,1024,2048").split(",")]
    kinds = [int(x) for x in os.environ.get("LZS_KINDS", "1,2").split(",")]
    mx = max(sizes)
    ctx = Context(max_block_bytes=64 << 20, max_batch_blocks=1, index_log2=20, arena_slots=16)
    dev = ctx.dev_alloc((mx << 20) + 4096)
    for kind in kinds:
        roots = np.array([r for r in range(1, 40 * mx) if segment_kind(r) == kind][:mx], np.uint32)
        ctx.corpus_fill(dev, roots, 1, mx, seg, 7, mixed=True)
        ctx.synchronize()
        for mib in sizes:
            n = mib << 20
            f = ctx.stream_block(4, 1, dev, n, n + 4096, [n])
            print(f"kind {kind} {mib:5d} MiB {(n + 261099) // 261100:6d} pieces -> ratio {len(f) / n:.3f}", flush=True)
    ctx.dev_free(dev)
    ctx.close()


if __name__ == "__main__":
    main()
