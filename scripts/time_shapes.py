#!/usr/bin/env python3
"""Timed shapes beside the headline (one JSON line each):
  jni_one_block   hdrf_reduce_block on host blocks (the JNI reduce0 shape: one 128 MiB block per
                  call, H2D included) and hdrf_reduce_batch of one resident block
  forced_cut      a full 128 MiB block in the forced-cut regime (0xFF bytes, 4 KiB random islands
                  every 9 MiB: chunks cut at 1,000,001 B, DN/DataDeduplicator.java:288-294) and an
                  all-0xFF block, through the same one-block call
Each block is checked against the oracle's chunk boundaries (offsets)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from hdrf_amd.corpus import corpus_roots          # noqa: E402
from hdrf_amd.lib import STAGES, Context          # noqa: E402
from oracle.oracle import chunk                   # noqa: E402

S = 128 << 20


def forced(seed):
    blk = np.full(S, 0xFF, np.uint8)
    isl = np.random.default_rng(seed).integers(0, 256, 4096 * 15, dtype=np.uint8)
    for i, o in enumerate(range(3 << 20, S - 4096, 9 << 20)):
        blk[o:o + 4096] = isl[(i % 15) * 4096:(i % 15 + 1) * 4096]
    return blk


def timed(ctx, fn, reps):
    fn()                                           # warm-up (allocations, first launch)
    ctx.stage_times(reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        r = fn()
    el = (time.perf_counter() - t0) / reps
    st = ctx.stage_times(reset=True)
    return r, el, {k.split("(")[0]: round(v / reps, 4) for k, v in zip(STAGES, st) if v > 0}


def main():
    ctx = Context(max_block_bytes=S, max_batch_blocks=1, index_log2=24, arena_slots=64, timing=1)
    roots = corpus_roots(77, 500000, 4, S >> 20)
    dev = ctx.dev_alloc(4 * S + 4096)
    ctx.corpus_fill(dev, roots, 4, S >> 20, 1 << 20, 77)
    host = [ctx.d2h(dev + b * S, S) for b in range(4)]
    out = []
    # JNI shape: host block per call (H2D + reduction + result read-back)
    ids = iter(range(10_000, 20_000))
    r, el, st = timed(ctx, lambda: ctx.reduce_block(host[0], next(ids)), 5)
    ok = np.array_equal(r["offsets"], chunk(host[0]))
    out.append({"shape": "jni_one_block_host", "block_bytes": S, "s_per_block": round(el, 5),
                "GB_s": round(S / el / 1e9, 2), "offsets_match_oracle": bool(ok), "stage_ms": st})
    r, el, st = timed(ctx, lambda: ctx.reduce_batch([dev + S], [S], [3 * S + 4096], [next(ids)]), 5)
    out.append({"shape": "one_resident_block", "block_bytes": S, "s_per_block": round(el, 5),
                "GB_s": round(S / el / 1e9, 2), "stage_ms": st})
    for name, blk in (("forced_cut_islands", forced(5)), ("all_0xff", np.full(S, 0xFF, np.uint8))):
        r, el, st = timed(ctx, lambda: ctx.reduce_block(blk, next(ids)), 3)
        ok = np.array_equal(r["offsets"], chunk(blk))
        out.append({"shape": name, "block_bytes": S, "chunks": int(len(r["offsets"])), "s_per_block": round(el, 5),
                    "GB_s": round(S / el / 1e9, 2), "offsets_match_oracle": bool(ok), "stage_ms": st})
    for o in out:
        print(json.dumps(o), flush=True)
    ctx.dev_free(dev)
    ctx.close()


if __name__ == "__main__":
    main()
