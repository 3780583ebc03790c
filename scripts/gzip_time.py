"""Times stream-mode compressor 5 (hdrf_stream_block codec 5) on one mixed-entropy block and
checks it against the host zlib (level 6, gzip wrapper) — run on the GPU box."""
import os
import sys
import time
import zlib

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from helpers import make_block  # noqa: E402
from hdrf_amd.lib import Context  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 32
n = mib << 20
kinds = ["text", "random", "binary", "lowent"]
a = np.concatenate([make_block(k, 5 + i, n // 4) for i, k in enumerate(kinds)])
ctx = Context(max_block_bytes=16 << 20, max_batch_blocks=8, index_log2=20, arena_slots=64)
dev = ctx.dev_alloc(n + 4096)
ctx.h2d(dev, a)
ctx.stream_block(5, 1, dev, 1 << 20, (1 << 20) + 4096, [1 << 20])     # warm-up
t = time.perf_counter()
f = ctx.stream_block(5, 2, dev, n, n + 4096, [n])
g = time.perf_counter() - t
t = time.perf_counter()
c = zlib.compressobj(6, zlib.DEFLATED, 31, 8)
z = c.compress(a.tobytes()) + c.flush()
h = time.perf_counter() - t
print({"mib": mib, "gpu_s": round(g, 3), "gpu_MB_s": round(n / g / 1e6, 1), "zlib_1core_s": round(h, 3),
       "zlib_MB_s": round(n / h / 1e6, 1), "ratio": round(n / len(f), 3), "equal_to_zlib": f == z}, flush=True)
