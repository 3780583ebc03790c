"""Progress probe for the GPU LZOP path: one stream_block_host + decode per size, timed."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_block  # noqa: E402
from hdrf_amd.lib import Context  # noqa: E402
from oracle.oracle import lzop_stream  # noqa: E402

ctx = Context(max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=16, arena_slots=16)
for kind in sys.argv[1].split(","):
    for n in [1, 32, 100, 1000, 49153, 245693, 600000]:
        d = make_block(kind, 11 + n, n)
        t = time.perf_counter()
        g = ctx.stream_block_host(3, 1, d, [n])
        t1 = time.perf_counter()
        ok = g == bytes(lzop_stream(d, [n]))
        r = bytes(ctx.stream_file_decode(3, g, n))
        print(f"{kind} n={n} enc {1e3 * (t1 - t):.1f} ms same={ok} dec {1e3 * (time.perf_counter() - t1):.1f} ms "
              f"roundtrip={r == d.tobytes()}", flush=True)
ctx.close()
