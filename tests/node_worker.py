"""One rank of tests/test_node.py::test_node_two_processes_gloo: a real torch.distributed rank
(gloo; both ranks share cuda:0) reducing its shard through hdrf_amd.node.NodeRank, then saving its
per-block results and views for the parent test to merge and check against the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCHED = [[2, 2], [1, 2], [2, 1]]
COMPRESSOR = int(os.environ.get("HDRF_NW_COMPRESSOR", "1"))   # 2: node-global Lz4Codec containers
CMAX = 1 << 20
SIZE = 600_000 if COMPRESSOR == 1 else 1_400_000


def blocks():
    from node_harness import mixed_blocks, plan
    seq = plan(SCHED)
    return seq, mixed_blocks(31, len(seq), SIZE)


def main(out):
    import torch.distributed as dist
    from hdrf_amd.lib import Context
    from hdrf_amd.node import NodeRank
    dist.init_process_group("gloo")
    r, G = dist.get_rank(), dist.get_world_size()
    seq, blks = blocks()
    ctx = Context(device=0, n_ranks=G, rank=r, container_max=CMAX, max_block_bytes=2 << 20, max_batch_blocks=4,
                  index_log2=20, arena_slots=128, compressor=COMPRESSOR)
    node = NodeRank(ctx)
    res = {}
    batches, mines, allp = [], [], []
    for j, per in enumerate(SCHED):
        mine = [gi for gi, (jj, rr, _) in enumerate(seq) if jj == j and rr == r]
        ptrs, lens, rd, ids = [], [], [], []
        for gi in mine:
            p = ctx.dev_alloc(len(blks[gi]) + 4096)
            ctx.h2d(p, blks[gi])
            ptrs.append(p); lens.append(len(blks[gi])); rd.append(len(blks[gi]) + 4096); ids.append(0x900 + gi)
        gbase, _ = node.batch_base(len(mine))
        batches.append((ptrs, lens, rd, ids, gbase))
        mines.append(mine)
        allp += ptrs

    def done(j):                       # the pipelined path (NodeRank.reduce_batches), as the bench runs it
        for i, gi in enumerate(mines[j]):
            b = ctx.batch_result(i)
            for k in ("offsets", "digests", "is_new", "container_id", "container_pos"):
                res[f"b{gi}_{k}"] = b[k]
            res[f"b{gi}_store"] = np.array([b["store_size"]])
            res[f"b{gi}_recipe"] = np.frombuffer(ctx.recipe(0x900 + gi), np.uint8)
    node.reduce_batches(batches, done)
    # the node read (DataConstructor over the node's one index): every rank takes part in every
    # read, the rank that reduced the block receives it
    for gi, (_, rr, _) in enumerate(seq):
        got = node.reconstruct_block(0x900 + gi, rr)
        if rr == r:
            res[f"b{gi}_read"] = got
        res[f"b{gi}_loc"] = node.last_loc
    for p in allp:
        ctx.dev_free(p)
    k, v = ctx.index_dump()
    res["index_keys"], res["index_vals"] = k, v
    res["alloc"] = np.frombuffer(ctx.allocator(), np.uint8)
    alloc = ctx.allocator()
    for t in range(3 if COMPRESSOR == 2 else 0):   # the Lz4Codec files this rank closed
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            f, closed = ctx.container(cid)
            if f is not None and closed:
                res[f"closed_{cid}"] = np.frombuffer(f, np.uint8)
    np.savez(os.path.join(out, f"rank{r}.npz"), **res)
    ctx.close()
    dist.destroy_process_group()


def check_outputs(out, G):
    from helpers import compare_block
    from oracle.oracle import Oracle
    seq, blks = blocks()
    ranks = [np.load(os.path.join(out, f"rank{r}.npz")) for r in range(G)]
    ora = Oracle(hasher=0, compressor=COMPRESSOR, max_size=CMAX)
    for gi, (_, r, _) in enumerate(seq):
        o = ora.reduce(blks[gi], 0x900 + gi)
        z = ranks[r]
        g = {k: z[f"b{gi}_{k}"] for k in ("offsets", "digests", "is_new", "container_id", "container_pos")}
        g["store_size"] = int(z[f"b{gi}_store"][0])
        compare_block(g, o, tag=f"global block {gi} on rank {r}")
        assert z[f"b{gi}_recipe"].tobytes() == ora.recipe(0x900 + gi)
        rd = z[f"b{gi}_read"]
        loc = z[f"b{gi}_loc"]
        offs = np.concatenate([[0], np.cumsum(loc[:, 2].astype(np.int64) - loc[:, 1])])
        badk = [k for k in range(len(loc)) if not np.array_equal(rd[offs[k]:offs[k + 1]], blks[gi][offs[k]:offs[k + 1]])]
        if badk:
            print("BAD chunks", gi, [(k, loc[k].tolist(), int(offs[k])) for k in badk[:10]])
            print("placers", np.bincount(loc[:, 3]))
        bad = np.nonzero(rd != blks[gi])[0] if rd.shape == blks[gi].shape else np.arange(1)
        assert bad.size == 0, (f"node read of global block {gi} on rank {r}: {bad.size} bytes differ, first at "
                               f"{bad[:8]}, len {rd.shape} vs {blks[gi].shape}, got {rd[bad[:8]] if rd.shape == blks[gi].shape else ''} "
                               f"want {blks[gi][bad[:8]]}")
    k = np.concatenate([z["index_keys"] for z in ranks])
    v = np.concatenate([z["index_vals"] for z in ranks])
    order = np.lexsort(k.T[::-1])
    ok, ov = ora.index_dump()
    assert np.array_equal(k[order], ok) and np.array_equal(v[order], ov), "node index differs"
    for z in ranks:
        assert z["alloc"].tobytes() == ora.allocator()
    alloc = ora.allocator()
    n_closed = 0
    # compressor 1 leaves each rank its own pieces of a shared container (the node read above
    # checks them); compressor 2 gathers every closed container into one file on its closer
    for t in range(3 if COMPRESSOR == 2 else 0):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, oc = ora.container(cid)
            if od is None or not oc:
                continue
            files = [z[f"closed_{cid}"] for z in ranks if f"closed_{cid}" in z.files]
            assert len(files) == 1 and files[0].tobytes() == od, f"closed container {cid:#x}"
            n_closed += 1
    return n_closed


if __name__ == "__main__":
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    main(sys.argv[1])
