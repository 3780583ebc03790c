#!/usr/bin/env python3
"""Index at steady state: the bench resets the index every step, so its load
factor stays <= 27 %.  Here the 2^27-entry table is first filled to a target load with random
digests (hdrf_index_load: Redis rows of an earlier life of the DataNode), then one config-2 batch
(32 x 128 MiB corpus blocks, 50 % dup) is reduced; reported per load: the index stages' times
(HIP events, serial batch), the measured probe lengths (hdrf_probe_stats: each chunk's distance
from its home slot) and linear probing's expected mean for comparison.  One JSON line per load."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hdrf_amd.corpus import corpus_roots          # noqa: E402
from hdrf_amd.lib import STAGES, Context          # noqa: E402

S, B, LOG2 = 128 << 20, 32, 27


def main():
    loads = [float(x) for x in (sys.argv[1:] or ["0", "0.3", "0.6", "0.8"])]
    ctx = Context(max_block_bytes=S, max_batch_blocks=B, index_log2=LOG2, arena_slots=512, timing=1)
    roots = corpus_roots(20251015, 500000, B, S >> 20)
    dev = ctx.dev_alloc(B * S + 4096)
    ctx.corpus_fill(dev, roots, B, S >> 20, 1 << 20, 20251015)
    ptrs = [dev + b * S for b in range(B)]
    rng = np.random.default_rng(7)
    for load in loads:
        ctx.reset()
        n = int(load * (1 << LOG2))
        t0 = time.perf_counter()
        step = 1 << 22
        for o in range(0, n, step):
            m = min(step, n - o)
            keys = rng.integers(0, 256, (m, ctx.H), dtype=np.uint8)
            vals = rng.integers(0, 256, (m, 11), dtype=np.uint8)
            vals[:, 0] = 1
            ctx.index_load(keys, vals)
        fill_s = time.perf_counter() - t0
        ctx.stage_times(reset=True)
        t0 = time.perf_counter()
        ctx.reduce_batch(ptrs, [S] * B, [B * S + 4096 - b * S for b in range(B)], list(range(B)))
        el = time.perf_counter() - t0
        st = dict(zip(STAGES, ctx.stage_times(reset=True)))
        psum, pmax, nch = ctx.probe_stats()
        a = n / (1 << LOG2)
        print(json.dumps({
            "load_before": round(a, 3), "prefill_rows": n, "prefill_s": round(fill_s, 1), "batch_chunks": nch,
            "probe_mean": round(psum / max(nch, 1), 3), "probe_max": pmax,
            "linear_probing_expected_mean_hit": round(0.5 * (1 + 1 / (1 - a)), 3),
            "linear_probing_expected_mean_miss": round(0.5 * (1 + 1 / (1 - a) ** 2), 3),
            "index_claim_ms": round(st["index_claim(idx_claim_kernel)"], 4),
            "index_apply_ms": round(st["index_apply(idx_apply_kernel)"], 4),
            "index_slow_decide_ms": round(st["index_slow_decide(idx_slow/decide)"], 4),
            "place_ms": round(st["place(place_kernel)"], 4), "batch_s": round(el, 4),
            "batch_GB_s": round(B * S / el / 1e9, 1)}), flush=True)
    ctx.dev_free(dev)
    ctx.close()


if __name__ == "__main__":
    main()
