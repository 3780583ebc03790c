"""Node-global ranks at the bench's batch shape in ONE process on one GPU (tests/node_harness.py
Loopback: G contexts, the X1/X2/X3 all-to-alls as region copies, no gloo or RCCL), pipelined as
NodeRank.reduce_batches runs them.  Measures what a rank's kernels cost per batch without the
time-sharing and host staging of the two-process rehearsal: run it under
`rocprofv3 --kernel-trace --stats` and divide each kernel's total by (batches x G).

  python scripts/node_loopback.py [--G 2] [--batches 4] [--batch 32] [--block-mib 128] [--check 1]

Prints one JSON line: wall time, the ranks' HIP-event stage times per batch (lib.STAGES), and, with
--check k, whether the first k global batches equal the oracle over the global block order
(DN/DataDeduplicator.java:124-204; every block's chunk offsets, digests, is_new and storeSize)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=2)
    ap.add_argument("--batches", type=int, default=4, help="global batches")
    ap.add_argument("--batch", type=int, default=32, help="blocks per rank per global batch")
    ap.add_argument("--block-mib", type=int, default=128)
    ap.add_argument("--index-log2", type=int, default=27)
    ap.add_argument("--check", type=int, default=0, help="global batches compared with the oracle")
    ap.add_argument("--seed", type=int, default=20251015)
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (the harness's exchange buffers)
    from hdrf_amd.corpus import corpus_roots
    from hdrf_amd.lib import STAGES
    from hdrf_amd.node import global_block
    from node_harness import Loopback, open_ranks

    G, B, nbat = a.G, a.batch, a.batches
    S, seg = a.block_mib << 20, 1 << 20
    spb = S // seg
    nb = B * nbat                                   # blocks per rank
    groots = corpus_roots(a.seed, 500000, nb * G, spb).reshape(nb * G, spb)
    ctxs = open_ranks(G, max_block_bytes=S, max_batch_blocks=B, index_log2=a.index_log2, arena_slots=512,
                      keep_recipes=1, timing=1)
    lb = Loopback(ctxs)
    devs, per_batch = [], []
    for r, c in enumerate(ctxs):
        mine = [global_block(L, r, G, B) for L in range(nb)]
        d = c.dev_alloc(nb * S + 4096)
        c.corpus_fill(d, groots[mine].reshape(-1), nb, spb, seg, a.seed)
        devs.append(d)
    total = nb * S + 4096
    for j in range(nbat):
        per = []
        for r in range(G):
            L0 = j * B
            per.append(([devs[r] + (L0 + i) * S for i in range(B)], [S] * B,
                        [total - (L0 + i) * S for i in range(B)],
                        [global_block(L0 + i, r, G, B) for i in range(B)]))
        per_batch.append(per)

    res = {}

    def done(j):
        if j < a.check:
            res[j] = [[ctxs[r].batch_result(i) for i in range(B)] for r in range(G)]

    for c in ctxs:
        c.stage_times(reset=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    lb.batches_pipelined(per_batch, done)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    stages = [c.stage_times(reset=True) for c in ctxs]
    per_rank_batch = {name: round(sum(st[i] for st in stages) / (G * nbat), 4) for i, name in enumerate(STAGES)}
    line = {"G": G, "global_batches": nbat, "blocks_per_rank_batch": B, "block_bytes": S,
            "wall_s": round(wall, 3), "logical_GB_s_one_gpu": round(G * nb * S / wall / 1e9, 2),
            "stage_ms_per_rank_batch": {k: v for k, v in per_rank_batch.items() if v > 0},
            "note": "all G ranks time-share one GPU; exchanges are device copies with a host sync each"}
    if a.check:
        from oracle.oracle import Oracle
        ora = Oracle()
        bad = 0
        checked = 0
        blocks = {}
        for j in range(a.check):
            for r in range(G):
                for i in range(B):
                    blocks[global_block(j * B + i, r, G, B)] = (r, j * B + i, res[j][r][i])
        order = sorted(blocks)
        data = [ctxs[blocks[g][0]].d2h(devs[blocks[g][0]] + blocks[g][1] * S, S) for g in order]
        thr = max(1, min(16, len(os.sched_getaffinity(0)) - 1))
        exp = ora.reduce_many_full(data, order, thr)
        for g, e in zip(order, exp):
            got = blocks[g][2]
            ok = (len(got["offsets"]) == len(e["offsets"]) and np.array_equal(got["offsets"], e["offsets"])
                  and np.array_equal(got["digests"], e["digests"]) and np.array_equal(got["is_new"], e["is_new"])
                  and got["store_size"] == e["store_size"])
            bad += not ok
            checked += 1
        line["oracle_check"] = {"blocks": checked, "mismatches": bad}
    print(json.dumps(line), flush=True)
    for c, d in zip(ctxs, devs):
        c.dev_free(d)
        c.close()


if __name__ == "__main__":
    main()
