"""Debug (HDRF_LIB_PATH=hdrf_amd/_build_dbg/libhdrf.so, built with -DHDRF_DEBUG_CHUNK): one config-4
batch (32 x 128 MiB mixed-entropy blocks); the repair give-ups and sequential fallbacks print from the
device.  Timing of the chunking stage per batch is printed too."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from hdrf_amd.corpus import corpus_roots
from hdrf_amd.lib import Context
S, spb = 128 << 20, 128
nb = 32
roots = corpus_roots(20251015, 500000, nb, spb)
ctx = Context(device=0, max_block_bytes=S, max_batch_blocks=32, index_log2=24, arena_slots=256, timing=1, compressor=1)
dev = ctx.dev_alloc(nb * S + 4096)
ctx.corpus_fill(dev, roots, nb, spb, 1 << 20, 20251015, mixed=True)
ptrs = [dev + b * S for b in range(nb)]
ctx.reduce_batch(ptrs, [S] * nb, [S + 4096] * nb, list(range(nb)))
ctx.synchronize()
print("stages", [round(x, 2) for x in ctx.stage_times(reset=True)], flush=True)
ctx.close()
