"""Debug: GPU stream-mode Lz4Codec (one write) vs the oracle, per kind and size; first difference."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_block  # noqa: E402
from hdrf_amd.lib import Context  # noqa: E402
from oracle.oracle import hadoop_lz4_stream  # noqa: E402

ctx = Context(max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=16, arena_slots=16)
bad = 0
for kind in ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"]:
    for n in [100, 4176, 65535, 70000, 200_000, 261_100, 600_000]:
        for seed in (3, 4):
            d = make_block(kind, seed + n, n)
            g = ctx.stream_block_host(4, 1, d, [n])
            o = hadoop_lz4_stream(d, [n])
            if g != o:
                bad += 1
                a = np.frombuffer(g, np.uint8); b = np.frombuffer(o, np.uint8)
                m = min(len(a), len(b))
                i = int(np.nonzero(a[:m] != b[:m])[0][0]) if (a[:m] != b[:m]).any() else m
                print(f"DIFF {kind} n={n} seed={seed}: len {len(a)} vs {len(b)}, first diff at {i}", flush=True)
print("bad", bad)
