"""Node-global index over G ranks (BASELINE config 3): G contexts that share one
index partitioned by digest prefix must reproduce, byte for byte, ONE sequential reduction of the
global block sequence (the oracle): chunk boundaries, digests, dedup decisions, storeSize,
container placement and bytes, every index value (nCopy + location), allocator and recipes.

GPU tests drive the ranks' HIP contexts on one device, either in one process (loopback copies
between the ranks' exchange buffers) or as real ranks over torch.distributed (gloo staging, the
same NodeRank code the 8-GPU bench runs over RCCL).  The CPU test covers the exchange plumbing
of hdrf_amd/node.py with world_size 2 on gloo."""
import os
import subprocess
import sys

import numpy as np
import pytest

from helpers import compare_block, make_block
from node_harness import mixed_blocks as _mixed_blocks, plan as _plan

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("G,hasher,sched", [
    (2, 0, [[2, 3], [3, 1], [1, 1]]),
    (3, 1, [[2, 2, 2], [1, 3, 2]]),
    (4, 0, [[1, 2, 1, 2], [2, 1, 1, 1]]),
    (8, 0, [[1, 2, 1, 1, 2, 1, 1, 1], [2, 1, 1, 2, 1, 1, 2, 1]]),    # the node's rank count
])
def test_node_loopback_matches_single_sequence(G, hasher, sched):
    import torch  # noqa: F401
    from node_harness import Loopback, assemble_containers, loopback_read, merged_index, open_ranks
    from oracle.oracle import Oracle

    cmax = 1 << 20                                   # small containers: many flushes across ranks
    seq = _plan(sched)
    blocks = _mixed_blocks(7 + G, len(seq), 700_000)
    ctxs = open_ranks(G, hasher=hasher, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=4,
                      index_log2=20, arena_slots=256)
    lb = Loopback(ctxs)
    ora = Oracle(hasher=hasher, compressor=1, max_size=cmax)
    devs = []
    pieces = []
    g = 0
    for j, per in enumerate(sched):
        per_rank, gidx = [], []
        for r, n in enumerate(per):
            ptrs, lens, rd, ids = [], [], [], []
            for i in range(n):
                blk = blocks[g + len(gidx)]
                gidx.append((r, i, g + len(gidx)))
                p = ctxs[r].dev_alloc(len(blk) + 4096)
                ctxs[r].h2d(p, blk)
                devs.append((ctxs[r], p))
                ptrs.append(p); lens.append(len(blk)); rd.append(len(blk) + 4096); ids.append(0x500 + 3 * (g + len(gidx) - 1))
            per_rank.append((ptrs, lens, rd, ids))
        lb.batch(per_rank)
        for r, i, gi in gidx:
            res = ctxs[r].batch_result(i)
            o = ora.reduce(blocks[gi], 0x500 + 3 * gi)
            compare_block(res, o, tag=f"G={G} batch {j} rank {r} block {i} (global {gi})")
            offs = res["offsets"]
            for k in np.nonzero(res["is_new"])[0]:
                a = int(offs[k - 1]) if k else 0
                pieces.append((int(res["container_id"][k]), int(res["container_pos"][k]),
                               blocks[gi][a:int(offs[k])].tobytes()))
        g += len(gidx)
    gk, gv = merged_index(ctxs)
    ok, ov = ora.index_dump()
    assert gk.shape == ok.shape and np.array_equal(gk, ok), "node index keys differ"
    bad = np.nonzero((gv != ov).any(axis=1))[0]
    assert bad.size == 0, f"index values differ at {bad[:5]}: {gv[bad[:3]]} vs {ov[bad[:3]]}"
    for c in ctxs:
        assert c.allocator() == ora.allocator(), "allocator differs"
    for gi in range(len(seq)):
        bid = 0x500 + 3 * gi
        owner = ctxs[seq[gi][1]]
        assert owner.recipe(bid) == ora.recipe(bid), f"recipe of global block {gi}"
    conts = assemble_containers(pieces)
    for cid, data in conts.items():
        od, _ = ora.container(cid)
        assert od is not None and od == data, f"container {cid:#x} bytes differ"
    alloc = ora.allocator()
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, _ = ora.container(cid)
            if od:
                assert cid in conts, f"container {cid:#x} missing"
    # the node read: every block rebuilt from the partitioned index and the ranks' arenas
    for gi in range(len(seq)):
        got = loopback_read(ctxs, seq[gi][1], 0x500 + 3 * gi)
        assert np.array_equal(got, blocks[gi]), f"node read of global block {gi}"
    from hdrf_amd.lib import HdrfError
    with pytest.raises(HdrfError):
        ctxs[0].reconstruct_block(0x500)                  # single-node read refused on G > 1
    for c, p in devs:
        c.dev_free(p)
    for c in ctxs:
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G,hasher,scan,depth", [(2, 1, "device", 3), (3, 0, "host", 2), (8, 1, "device", 4),
                                                 (4, 0, "device", 5)])
def test_node_loopback_pipelined_matches_single_sequence(G, hasher, scan, depth, monkeypatch):
    """The pipelined phase order (the fronts of `depth` batches launched ahead on the chunking, SHA
    and aggregation streams, each rank's slot reused only after its previous batch's back phases;
    the back phases on stream B, the arena copy on B2; the allocator scan on the device over the
    all-gathered packed descriptors, or on the host) gives the same bytes as the oracle."""
    import torch  # noqa: F401
    from node_harness import Loopback, merged_index, open_ranks
    from oracle.oracle import Oracle
    monkeypatch.setenv("HDRF_GX_DEPTH", str(depth))

    cmax = 1 << 20
    sched = [([2, 1, 2] * 3)[:G], ([1, 2, 1] * 3)[:G], ([2, 2, 1] * 3)[:G], ([1, 1, 2] * 3)[:G]]
    seq = _plan(sched)
    blocks = _mixed_blocks(41 + G, len(seq), 600_000)
    ctxs = open_ranks(G, hasher=hasher, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=4,
                      index_log2=20, arena_slots=256)
    lb = Loopback(ctxs)
    ora = Oracle(hasher=hasher, compressor=1, max_size=cmax)
    devs, per_batch, where = [], [], []
    g = 0
    for j, per in enumerate(sched):
        pr, wj = [], []
        for r, n in enumerate(per):
            ptrs, lens, rd, ids = [], [], [], []
            for i in range(n):
                blk = blocks[g]
                p = ctxs[r].dev_alloc(len(blk) + 4096)
                ctxs[r].h2d(p, blk)
                devs.append((ctxs[r], p))
                ptrs.append(p); lens.append(len(blk)); rd.append(len(blk) + 4096); ids.append(0x700 + g)
                wj.append((r, i, g))
                g += 1
            pr.append((ptrs, lens, rd, ids))
        per_batch.append(pr)
        where.append(wj)

    def done(j):
        for r, i, gi in where[j]:
            compare_block(ctxs[r].batch_result(i), ora.reduce(blocks[gi], 0x700 + gi),
                          tag=f"pipelined G={G} batch {j} rank {r} block {i}")
    assert int(ctxs[0].gx_layout().depth) == depth
    lb.batches_pipelined(per_batch, done, scan=scan)
    from node_harness import loopback_read
    for wj in where:
        for r, i, gi in wj:
            got = loopback_read(ctxs, r, 0x700 + gi)
            bad = np.nonzero(got != blocks[gi])[0]
            assert bad.size == 0, f"pipelined node read of block {gi}: {bad.size} bytes differ, first {bad[:8]}"
    gk, gv = merged_index(ctxs)
    ok, ov = ora.index_dump()
    assert np.array_equal(gk, ok) and np.array_equal(gv, ov), "node index differs"
    for c in ctxs:
        assert c.allocator() == ora.allocator()
    for c, p in devs:
        c.dev_free(p)
    for c in ctxs:
        c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("G,pipelined", [(3, False), (8, True)])
def test_node_loopback_compressor2_matches_single_sequence(G, pipelined):
    """The reference's default mode (compressor 2, DN/DataNode.java:438) on a node-global index:
    a container closed by rank s whose head earlier ranks wrote is gathered on s and rewritten as
    one Lz4Codec file (DN/DataDeduplicator.java:748-797).  Every closed container's file equals the
    oracle's, byte for byte, on the rank that closed it; blocks, index and allocator as before."""
    import torch  # noqa: F401
    from node_harness import Loopback, merged_index, open_ranks
    from oracle.oracle import Oracle

    cmax = 1 << 20                                   # the smallest container that holds a maximal chunk
    sched = [([2, 1, 2] * 3)[:G], ([1, 2, 1] * 3)[:G], ([2, 2, 1] * 3)[:G], ([1, 1, 2] * 3)[:G]]
    seq = _plan(sched)
    blocks = _mixed_blocks(61 + G, len(seq), 1_400_000)
    ctxs = open_ranks(G, hasher=0, compressor=2, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=4,
                      index_log2=20, arena_slots=256)
    lb = Loopback(ctxs)
    ora = Oracle(hasher=0, compressor=2, max_size=cmax)
    devs, per_batch, where = [], [], []
    g = 0
    for per in sched:
        pr, wj = [], []
        for r, n in enumerate(per):
            ptrs, lens, rd, ids = [], [], [], []
            for i in range(n):
                blk = blocks[g]
                p = ctxs[r].dev_alloc(len(blk) + 4096)
                ctxs[r].h2d(p, blk)
                devs.append((ctxs[r], p))
                ptrs.append(p); lens.append(len(blk)); rd.append(len(blk) + 4096); ids.append(0x900 + g)
                wj.append((r, i, g))
                g += 1
            pr.append((ptrs, lens, rd, ids))
        per_batch.append(pr)
        where.append(wj)

    def done(j):
        for r, i, gi in where[j]:
            compare_block(ctxs[r].batch_result(i), ora.reduce(blocks[gi], 0x900 + gi),
                          tag=f"c2 G={G} batch {j} rank {r} block {i}")
    if pipelined:
        lb.batches_pipelined(per_batch, done)
    else:
        for j, pr in enumerate(per_batch):
            lb.batch(pr)
            done(j)
    gk, gv = merged_index(ctxs)
    ok, ov = ora.index_dump()
    assert np.array_equal(gk, ok) and np.array_equal(gv, ov), "node index differs"
    alloc = ora.allocator()
    n_closed = 0
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, oc = ora.container(cid)
            if od is None or not oc:
                continue
            files = [f for f, closed in (c.container(cid) for c in ctxs) if closed]
            assert len(files) == 1, f"container {cid:#x} closed on {len(files)} ranks"
            assert files[0] == od, f"container {cid:#x}: Lz4Codec file differs ({len(files[0])} vs {len(od)} B)"
            n_closed += 1
    assert n_closed >= 6, f"only {n_closed} containers closed"
    assert getattr(lb, "moved", 0) > 0, "no head piece was gathered"
    st = [c.stats() for c in ctxs]
    assert sum(x["closed_containers"] for x in st) == n_closed
    for c, p in devs:
        c.dev_free(p)
    for c in ctxs:
        c.close()


def _load_ranks(ctxs, blocks_per_rank, id0):
    per_rank, devs = [], []
    for r, blks in enumerate(blocks_per_rank):
        ptrs, lens, rd, ids = [], [], [], []
        for i, blk in enumerate(blks):
            p = ctxs[r].dev_alloc(len(blk) + 4096)
            ctxs[r].h2d(p, blk)
            devs.append((ctxs[r], p))
            ptrs.append(p); lens.append(len(blk)); rd.append(len(blk) + 4096); ids.append(id0 + 16 * r + i)
        per_rank.append((ptrs, lens, rd, ids))
    return per_rank, devs


@pytest.mark.gpu
def test_node_owner_table_full_is_a_clean_error():
    """an owner whose index partition fills during hdrf_gx_owner (device error 2; the
    failing records' owner slots are never written) must not touch the table again.  Its X2
    responses are "not created, not the minimum" for every record, so no source designates a
    chunk or sends an X3 location, and hdrf_gx_place reports HDRF_E_CAPACITY ("index table full").
    The device keeps working: a fresh node on the same GPU reduces correctly afterwards."""
    import torch
    from node_harness import Loopback, open_ranks
    from hdrf_amd.lib import HdrfError
    G = 2
    blocks = [[make_block("random", 900 + 2 * r + i, 700_000) for i in range(2)] for r in range(G)]
    ctxs = open_ranks(G, container_max=1 << 20, max_block_bytes=4 << 20, max_batch_blocks=4, index_log2=10,
                      arena_slots=64)
    lb = Loopback(ctxs)
    per_rank, devs = _load_ranks(ctxs, blocks, 0x900)
    c1 = [ctxs[r].gx_front(*per_rank[r], 2 * r, lb.x1s[r].data_ptr()) for r in range(G)]
    r1 = lb._a2a(lb.x1s, lb.x1r, c1, lb.w[0])
    assert all(sum(r1[d]) > 1024 for d in range(G)), "each owner must receive more digests than its 1024 entries"
    for d in range(G):
        ctxs[d].gx_owner(lb.x1r[d].data_ptr(), r1[d], lb.x2s[d].data_ptr())
    torch.cuda.synchronize()
    for d in range(G):
        x2 = lb.x2s[d].view(G, lb.cap, 2)
        for s_ in range(G):
            assert int(x2[s_, :r1[d][s_]].abs().sum()) == 0, "responses after a full table must decide nothing"
    lb._a2a(lb.x2s, lb.x2r, r1, lb.w[1])
    for r in range(G):
        ctxs[r].gx_decide(lb.x2r[r].data_ptr())
    a = None
    for r in range(G):
        a = ctxs[r].gx_flush(a)
    with pytest.raises(HdrfError) as ei:
        ctxs[0].gx_place(a, lb.x3s[0].data_ptr())
    assert ei.value.code == -4 and "index table full" in str(ei.value), str(ei.value)
    torch.cuda.synchronize()
    for c, p in devs:
        c.dev_free(p)
    for c in ctxs:
        c.close()
    # the GPU is healthy: a node with a large enough partition reduces the same blocks exactly
    from oracle.oracle import Oracle
    ctxs = open_ranks(G, container_max=1 << 20, max_block_bytes=4 << 20, max_batch_blocks=4, index_log2=16,
                      arena_slots=64)
    lb = Loopback(ctxs)
    per_rank, devs = _load_ranks(ctxs, blocks, 0x900)
    lb.batch(per_rank)
    ora = Oracle(max_size=1 << 20)
    for r in range(G):
        for i in range(2):
            compare_block(ctxs[r].batch_result(i), ora.reduce(blocks[r][i], 0x900 + 16 * r + i), tag=f"after error r{r} b{i}")
    for c, p in devs:
        c.dev_free(p)
    for c in ctxs:
        c.close()


@pytest.mark.gpu
def test_node_compress_step_is_enforced_and_idempotent():
    """under compressor 2 on a node-global context, hdrf_gx_commit refuses a batch whose
    closed containers were not compressed (their reads would come from an unwritten compressed
    arena), and a second hdrf_gx_compress changes nothing (file lengths and closed_file_bytes stay
    those of one pass)."""
    import torch  # noqa: F401
    from node_harness import Loopback, open_ranks
    from hdrf_amd.lib import HdrfError
    from oracle.oracle import Oracle
    G, cmax = 2, 1 << 20
    blocks = [[make_block("text", 950 + 2 * r + i, 1_500_000) for i in range(2)] for r in range(G)]
    ctxs = open_ranks(G, compressor=2, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=4,
                      index_log2=18, arena_slots=64)
    lb = Loopback(ctxs)
    per_rank, devs = _load_ranks(ctxs, blocks, 0xA00)
    c1 = [ctxs[r].gx_front(*per_rank[r], 2 * r, lb.x1s[r].data_ptr()) for r in range(G)]
    r1 = lb._a2a(lb.x1s, lb.x1r, c1, lb.w[0])
    for d in range(G):
        ctxs[d].gx_owner(lb.x1r[d].data_ptr(), r1[d], lb.x2s[d].data_ptr())
    lb._a2a(lb.x2s, lb.x2r, r1, lb.w[1])
    for r in range(G):
        ctxs[r].gx_decide(lb.x2r[r].data_ptr())
    a = None
    for r in range(G):
        a = ctxs[r].gx_flush(a)
    c3 = [ctxs[r].gx_place(a, lb.x3s[r].data_ptr()) for r in range(G)]
    r3 = lb._a2a(lb.x3s, lb.x3r, c3, lb.w[2])
    closers = [r for r in range(G) if ctxs[r].stats()["closed_containers"] > 0]
    assert closers, "some rank must close a container"
    with pytest.raises(HdrfError) as ei:
        ctxs[closers[0]].gx_commit(lb.x3r[closers[0]].data_ptr(), r3[closers[0]])
    assert ei.value.code == -1 and "hdrf_gx_compress" in str(ei.value)
    lb._compress()
    before = [ctxs[r].stats()["closed_file_bytes"] for r in range(G)]
    for r in range(G):
        assert ctxs[r].gx_compress() == 0, "a second compress is a no-op"
    assert [ctxs[r].stats()["closed_file_bytes"] for r in range(G)] == before
    for d in range(G):
        ctxs[d].gx_commit(lb.x3r[d].data_ptr(), r3[d])
    ora = Oracle(compressor=2, max_size=cmax)
    for r in range(G):
        for i in range(2):
            compare_block(ctxs[r].batch_result(i), ora.reduce(blocks[r][i], 0xA00 + 16 * r + i), tag=f"c2 r{r} b{i}")
    alloc, n_closed = ora.allocator(), 0
    for t in range(3):
        for cid in range(t << 22, int.from_bytes(alloc[3 * t:3 * t + 3], "big") + 1):
            od, oc = ora.container(cid)
            if od is not None and oc:
                files = [f for f, closed in (c.container(cid) for c in ctxs) if closed]
                assert files == [od], f"container {cid:#x}: Lz4Codec file differs"
                n_closed += 1
    assert n_closed > 0
    for c, p in devs:
        c.dev_free(p)
    for c in ctxs:
        c.close()


@pytest.mark.gpu
def test_node_context_rejects_single_node_calls():
    from hdrf_amd.lib import Context, HdrfError
    ctx = Context(n_ranks=2, rank=1, max_block_bytes=1 << 20, max_batch_blocks=2, index_log2=16, arena_slots=16,
                  container_max=1 << 21)
    with pytest.raises(HdrfError):
        ctx.reduce_block(make_block("random", 1, 5000), 1)
    with pytest.raises(HdrfError):                      # phases out of order
        ctx.gx_decide(0)
    ctx.close()


@pytest.mark.gpu
def test_node_two_processes_gloo(tmp_path):
    """Two real ranks (one process each, both on cuda:0, gloo staging) through NodeRank."""
    out = str(tmp_path)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29631", os.path.join(ROOT, "tests", "node_worker.py"), out]
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests"))
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    from node_worker import check_outputs
    check_outputs(out, 2)


@pytest.mark.gpu
def test_node_two_processes_gloo_compressor2(tmp_path):
    """Two real ranks over gloo with compressor 2: the head pieces cross processes (batched
    isend/irecv in NodeRank._compress) and every closed container's Lz4Codec file is the oracle's."""
    out = str(tmp_path)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29633", os.path.join(ROOT, "tests", "node_worker.py"), out]
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.path.join(ROOT, "tests"), HDRF_NW_COMPRESSOR="2")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    os.environ["HDRF_NW_COMPRESSOR"] = "2"
    try:
        import importlib
        import node_worker
        importlib.reload(node_worker)
        assert node_worker.check_outputs(out, 2) >= 4
    finally:
        del os.environ["HDRF_NW_COMPRESSOR"]
        importlib.reload(node_worker)


def test_container_pieces_plan_cpu():
    """hdrf_amd.node.ContainerPieces: the head pieces a closer needs, from allocator states only
    (three ranks; range 0's container 0 spans ranks 0-2 and closes on rank 2; range 1's closes on
    the rank that opened it; range 2 idle)."""
    from hdrf_amd.node import ContainerPieces

    def st(ids, curs, exists):
        w = np.zeros(32, np.uint32)
        w[0:3], w[4:7], w[18:21] = ids, curs, exists
        return w.view(np.uint8)

    t1, t2 = 1 << 22, 2 << 22
    ains = [st([0, t1, t2], [0, 0, 0], [0, 0, 0]), st([0, t1 + 1, t2], [100, 5, 0], [1, 1, 0]),
            st([0, t1 + 1, t2], [250, 9, 0], [1, 1, 0])]
    aouts = [st([0, t1 + 1, t2], [100, 5, 0], [1, 1, 0]), st([0, t1 + 1, t2], [250, 9, 0], [1, 1, 0]),
             st([1, t1 + 1, t2], [40, 9, 0], [1, 1, 0])]
    cp = ContainerPieces(3)
    x = cp.batch(ains, aouts)
    assert sorted(x) == [(0, 2, 0, 0, 100), (1, 2, 0, 100, 250)]
    assert cp.open[0] == (1, [(2, 0, 40)])
    # range 1: rank 0 closed t1 itself (no transfer), ranks 1 continued t1 + 1
    assert cp.open[1] == (t1 + 1, [(0, 0, 5), (1, 5, 9)])
    # next batch: rank 0 closes t1 + 1 -> rank 1's piece [5, 9) moves, rank 0's own [0, 5) stays
    ains2 = [st([1, t1 + 1, t2], [40, 9, 0], [1, 1, 0])] * 3
    aouts2 = [st([1, t1 + 2, t2], [40, 3, 0], [1, 1, 0])] + [st([1, t1 + 2, t2], [40, 3, 0], [1, 1, 0])] * 2
    x2 = cp.batch(ains2, [aouts2[0], ains2[1], ains2[2]])
    assert x2 == [(1, 0, t1 + 1, 5, 9)]


def test_exchange_gloo_cpu_world2():
    """hdrf_amd.node.Exchange on CPU tensors, world_size 2 over gloo: counts, variable regions and
    the allocator hand-off chain."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", "29641", os.path.join(ROOT, "tests", "exchange_worker.py")]
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("exchange ok") == 2, r.stdout[-2000:]


@pytest.mark.gpu
def test_exchange_rccl_gpu():
    """The RCCL branch of hdrf_amd.node.Exchange (backend "nccl" is RCCL on ROCm) on device
    tensors: counts (all_to_all_single), variable-length record regions (list all_to_all), the
    allocator hand-off (broadcast; send/recv need a second rank) and the all-gather of scan
    descriptors.  One GPU here, so world size 1 (every exchange is the rank's own region); the
    8-GPU node run is the driver's."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "1", "--master-addr", "127.0.0.1",
           "--master-port", "29643", os.path.join(ROOT, "tests", "exchange_worker.py")]
    env = dict(os.environ, PYTHONPATH=ROOT, HDRF_XW_BACKEND="nccl")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.count("exchange ok 0 nccl") == 1, r.stdout[-2000:]


@pytest.mark.gpu
def test_node_bench_rehearsal_two_ranks_one_device(tmp_path):
    """The N > 1 bench line (two ranks sharing cuda:0 over gloo, HDRF_BENCH_SAME_DEVICE=1: a rehearsal
    of --gpus 2, not a measurement) carries non-zero times for every stream of the node-global
    pipeline (front: chunking / SHA / local aggregation; back: owner .. commit with the device
    allocator scan; arena copy), and its dedup result equals the 1-rank line's on the same global
    corpus (rank-major global batches are the global block order)."""
    import json
    common = ["--block-mib", "16", "--batch", "4", "--steps", "1", "--warmup", "1", "--index-log2", "22",
              "--arena-slots", "128", "--no-cpu", "--no-sub", "--no-alone"]
    env = dict(os.environ, HDRF_BENCH_SAME_DEVICE="1", PYTHONPATH=ROOT)
    r2 = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr",
                         "127.0.0.1", "--master-port", "29651", os.path.join(ROOT, "bench.py"), "--gpus", "2",
                         "--blocks", "12"] + common, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    l2 = json.loads([x for x in r2.stdout.splitlines() if x.startswith("{")][-1])
    r1 = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--blocks", "24"] + common, cwd=ROOT,
                        env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True, text=True, timeout=400)
    assert r1.returncode == 0, r1.stdout[-3000:] + r1.stderr[-3000:]
    l1 = json.loads([x for x in r1.stdout.splitlines() if x.startswith("{")][-1])
    print(json.dumps(l2["roofline"]["chains_ms_per_batch"]), l2["roofline"].get("front_period_ms"))
    print(json.dumps(l2.get("node_back_ms_per_batch")))
    for k in ("stored_bytes", "chunks", "logical_bytes"):
        assert l2["dedup"][k] == l1["dedup"][k], (k, l2["dedup"][k], l1["dedup"][k])
    chains = l2["roofline"]["chains_ms_per_batch"]
    assert set(chains) == {"W: chunking", "A: SHA", "X: local aggregation", "B: back (owner .. commit + exchanges)",
                           "B2: arena copy"}
    assert all(v > 0 for v in chains.values()), chains
    st = l2["stages"]
    for k in ("place(place_kernel)", "flush(flush_kernel)", "gx_owner(own_claim..own_finish)",
              "gx_alloc_scan(gx_scan_kernel)", "gx_commit(own_commit)", "gx_local(scratch claim/apply/decide + gx_emit)"):
        assert st[k]["ms_per_step"] > 0, (k, st[k])
    assert l2["roofline"]["frac"] > 0 and l2["roofline"]["front_period_ms"] > 0


@pytest.mark.gpu
@pytest.mark.timeout(900)
def test_node_loopback_bench_shape_two_ranks():
    """Node-global ranks at the bench's exact batch shape (scripts/node_loopback.py: G = 2 contexts
    on one device as the bench opens them — 32 x 128 MiB blocks per rank per global batch, index
    2^27, 512 arena slots, recipes, timing — the bench's global corpus sharded rank-major, pipelined
    as NodeRank.reduce_batches): both global batches, 64 blocks of 128 MiB, equal the oracle over the
    global block order chunk for chunk (offsets, digests, is_new, storeSize)."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "node_loopback.py"), "--G", "2", "--batches",
                        "2", "--check", "2"], cwd=ROOT, env=dict(os.environ, PYTHONPATH=ROOT), capture_output=True,
                       text=True, timeout=850)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    print(json.dumps(line))
    assert line["oracle_check"] == {"blocks": 128, "mismatches": 0}, line["oracle_check"]


@pytest.mark.gpu
@pytest.mark.parametrize("G,compressor,scan", [(2, 1, "device"), (3, 2, "device"), (2, 1, "host")])
def test_node_loopback_reset_async_generations(G, compressor, scan, monkeypatch):
    """Node-global hdrf_reset_async (bench.py's primed N > 1 steps): three generations of two or three
    global batches, each started with hdrf_reset_async on every rank before its first front while the
    previous generation's batches are still in the pipeline.  Every block equals a fresh oracle per
    generation (the switch is made by the first new batch's owner phase: the next epoch, the node's
    allocator re-seeded after the old commits and arena copies); after the last generation the
    merged index and the allocator are that generation's oracle's."""
    import torch  # noqa: F401
    from node_harness import Loopback, merged_index, open_ranks
    from oracle.oracle import Oracle
    monkeypatch.setenv("HDRF_GX_DEPTH", "3")
    cmax = 1 << 20
    gens_sched = [[[2] * G, [1] * G, [2] * G], [[1] * G, [2] * G], [[2] * G, [1] * G, [1] * G]]
    ctxs = open_ranks(G, compressor=compressor, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=4,
                      index_log2=20, arena_slots=256)
    lb = Loopback(ctxs)
    devs, per_batch, where, starts = [], [], [], []
    oras, blocks_of = [], []
    for q, sched in enumerate(gens_sched):
        seq = _plan(sched)
        blocks = _mixed_blocks(61 + q, len(seq), 500_000)
        blocks_of.append(blocks)
        oras.append(Oracle(compressor=compressor, max_size=cmax))
        starts.append(len(per_batch))
        g = 0
        for per in sched:
            pr, wj = [], []
            for r, n in enumerate(per):
                ptrs, lens, rd, ids = [], [], [], []
                for i in range(n):
                    blk = blocks[g]
                    p = ctxs[r].dev_alloc(len(blk) + 4096)
                    ctxs[r].h2d(p, blk)
                    devs.append((ctxs[r], p))
                    ptrs.append(p); lens.append(len(blk)); rd.append(len(blk) + 4096); ids.append(0x900 + g)
                    wj.append((q, r, i, g))
                    g += 1
                pr.append((ptrs, lens, rd, ids))
            per_batch.append(pr)
            where.append(wj)

    def done(j):
        for q, r, i, gi in where[j]:
            compare_block(ctxs[r].batch_result(i), oras[q].reduce(blocks_of[q][gi], 0x900 + gi),
                          tag=f"generation {q} batch {j} rank {r} block {i}")
    lb.batches_pipelined(per_batch, done, scan=scan, gens=starts)
    gk, gv = merged_index(ctxs)
    ok, ov = oras[-1].index_dump()
    assert np.array_equal(gk, ok) and np.array_equal(gv, ov), "node index after the last generation differs"
    for r, c in enumerate(ctxs):
        assert c.allocator() == oras[-1].allocator()
        assert c.stats()["blocks"] == sum(per[r] for per in gens_sched[-1]), "the totals are the last generation's"
    for c, p in devs:
        c.dev_free(p)
    for c in ctxs:
        c.close()
