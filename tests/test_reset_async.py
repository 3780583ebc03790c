"""hdrf_reset_async: a fresh DataNode from the next submit on, without draining the batches in flight
(the bench's back-to-back steps).  The batches submitted before it complete against the old state,
those after it against a fresh index, allocator, containers and recipes — each sequence equal to its
own oracle run, for compressor 1 and 2, across several resets (epochs) and a forced epoch wrap; with
durable containers (the streaming DataNode of BASELINE config 5) every generation's drained files
equal its own oracle's containers while the slot rings wrap across the generations."""
import numpy as np
import pytest

from helpers import compare_block, compare_state, make_block
from hdrf_amd.corpus import corpus_block_host, corpus_roots
from hdrf_amd.lib import Context, HdrfError
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _blocks(seed, n, spb=4, mixed=False):
    roots = corpus_roots(seed, 500000, n, spb)
    return [corpus_block_host(seed, roots, b, spb, 1 << 18, mixed=mixed) for b in range(n)]


@pytest.mark.parametrize("compressor", [1, 2])
def test_reset_async_between_pipelined_sequences(compressor):
    cmax = 1 << 20
    seqs = [_blocks(60 + i, 9, mixed=compressor == 2) for i in range(3)]
    ctx = Context(container_max=cmax, compressor=compressor, max_block_bytes=1 << 20, max_batch_blocks=3,
                  index_log2=18, arena_slots=64)
    size = len(seqs[0][0])
    dev = ctx.dev_alloc(size * 27 + 4096)
    ctx.h2d(dev, np.concatenate([b for s in seqs for b in s]))
    total = size * 27 + 4096
    pend = []                      # (sequence, first block) of the batches in flight, FIFO
    oras = [Oracle(compressor=compressor, max_size=cmax) for _ in seqs]
    last_ids = None
    for q in range(3):
        ctx.reset_async()          # batches of the previous sequence are still in flight here
        for b0 in range(0, 9, 3):
            g0 = q * 9 + b0
            ctx.submit_batch([dev + (g0 + i) * size for i in range(3)], [size] * 3,
                             [total - (g0 + i) * size for i in range(3)], [0x600 + b0 + i for i in range(3)])
            pend.append((q, b0))
            if len(pend) == 4:
                qq, bb = pend.pop(0)
                ctx.wait_batch()
                for i in range(3):
                    compare_block(ctx.batch_result(i), oras[qq].reduce(seqs[qq][bb + i], 0x600 + bb + i),
                                  tag=f"seq {qq} block {bb + i}")
        last_ids = [0x600 + i for i in range(9)]
    while pend:
        qq, bb = pend.pop(0)
        ctx.wait_batch()
        for i in range(3):
            compare_block(ctx.batch_result(i), oras[qq].reduce(seqs[qq][bb + i], 0x600 + bb + i),
                          tag=f"seq {qq} block {bb + i}")
    compare_state(ctx, oras[2], last_ids, tag="after the last reset")
    st = ctx.stats()
    assert st["blocks"] == 9, st            # the totals are the last generation's
    ctx.dev_free(dev)
    ctx.close()


def test_reset_async_epoch_wrap_and_refusals():
    """More than 255 generations: the epoch wraps and the table is cleared on the index stream, in
    order."""
    blocks = _blocks(77, 4)
    ctx = Context(container_max=1 << 20, max_block_bytes=1 << 20, max_batch_blocks=2, index_log2=16, arena_slots=32)
    size = len(blocks[0])
    dev = ctx.dev_alloc(size * 4 + 4096)
    ctx.h2d(dev, np.concatenate(blocks))
    ptrs = [dev + i * size for i in range(4)]
    rd = [size * (4 - i) + 4096 for i in range(4)]
    inflight = 0
    for gen in range(260):
        ctx.reset_async()                             # two or three batches of earlier generations in flight
        while inflight > 2:
            ctx.wait_batch()
            inflight -= 1
        ctx.submit_batch(ptrs[:2], [size] * 2, rd[:2], [1, 2])
        ctx.submit_batch(ptrs[2:], [size] * 2, rd[2:], [3, 4])
        inflight += 2
    while inflight:
        ctx.wait_batch()
        inflight -= 1
    ora = Oracle(max_size=1 << 20)
    for i, b in enumerate(blocks):
        ora.reduce(b, i + 1)
    compare_state(ctx, ora, [1, 2, 3, 4], tag="after 260 generations")
    ctx.dev_free(dev)
    ctx.close()


def _durable_blocks(seed, n, size=2 << 20):
    """~3/4 new random bytes per block (the slot rings wrap), the rest cross-block duplicates."""
    rng = np.random.default_rng(seed)
    base = [make_block(k, seed + i, 600_000) for i, k in enumerate(["random", "text", "binary"])]
    d = size // 8
    return [np.concatenate([base[int(rng.integers(3))][int(rng.integers(0, 200_000)):][:d] for _ in range(2)] +
                           [make_block("random", seed + 100 + i, size - 2 * d)]) for i in range(n)]


def _apply(disk, events):
    for cid, closed, off, data in events:
        if off == 0:
            disk[cid] = (bytearray(data), bool(closed))
        else:
            f = disk.get(cid, (bytearray(), False))[0]
            assert len(f) == off, f"append to {cid} at {off}, file has {len(f)}"
            f[off:] = data
            disk[cid] = (f, bool(closed))


def _check_files(disk, ora, tag):
    alloc = ora.allocator()
    n = 0
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, oc = ora.container(cid)
            if od is None:
                continue
            n += 1
            assert cid in disk and bytes(disk[cid][0]) == bytes(od) and disk[cid][1] == oc, f"{tag}: container {cid}"
    assert n == len(disk), f"{tag}: {len(disk)} files drained, the oracle has {n}"
    return n


@pytest.mark.parametrize("compressor,ngen,nblk,slots", [(1, 3, 16, 80), (2, 3, 16, 80), (1, 16, 2, 80)])
def test_reset_async_durable_generations(compressor, ngen, nblk, slots):
    """Durable containers: generations of host blocks submitted three deep, hdrf_reset_async
    between them with the previous generation's batches in flight, a drain after every completed
    batch.  Each generation's blocks and drained files equal its own oracle run, and the rings of
    slots / 4 per range wrap across the generations (the new generation continues each ring past
    the old open container).  Two-block generations put two generation switches in flight at once
    (each holds one more slot per ring until it is waited for)."""
    cmax = 1 << 20
    gens = [_durable_blocks(91 + 7 * g + compressor, nblk) for g in range(ngen)]
    ctx = Context(compressor=compressor, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=1,
                  index_log2=20, arena_slots=slots, retain_containers=1)
    oras = [Oracle(compressor=compressor, max_size=cmax) for _ in gens]
    disks = [{} for _ in gens]
    pend = []

    def complete():
        g, b = pend.pop(0)
        ctx.wait_batch()
        compare_block(ctx.batch_result(0), oras[g].reduce(gens[g][b], 0x700 + b), tag=f"gen {g} block {b}")
        _apply(disks[g], ctx.drain_containers(buf_bytes=1 << 20))

    for g, blocks in enumerate(gens):
        ctx.reset_async()                              # the previous generation's batches still in flight
        for b, blk in enumerate(blocks):
            ctx.submit_host([blk.ctypes.data], [len(blk)], [0x700 + b])
            pend.append((g, b))
            if len(pend) == 3:
                complete()
    while pend:
        complete()
    assert ctx.drain_containers() == []
    total = sum(_check_files(disks[g], oras[g], f"generation {g}") for g in range(ngen))
    assert total > slots - slots // 4, "the rings of slots / 4 per range must have wrapped"
    compare_state(ctx, oras[-1], [0x700 + b for b in range(nblk)], tag=f"durable generations c{compressor}",
                  containers=False)
    ctx.close()


def test_reset_async_durable_undrained_refused():
    """The wait for the new generation's first batch fails when an old container was not handed out
    (the new generation reuses the container ids) and leaves that batch in flight: after
    hdrf_drain_containers the same wait completes it, the old generation's files equal its oracle's
    and the new generation's block and state equal a fresh oracle's.  A view that must complete such a
    batch anyway drops the old containers, reports it, and the context works again after hdrf_reset."""
    cmax = 1 << 20
    blocks = _durable_blocks(97, 4)
    ctx = Context(container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=20, arena_slots=64,
                  retain_containers=1)
    ctx.reset_async()
    ctx.submit_host([blocks[0].ctypes.data], [len(blocks[0])], [1])
    ctx.reset_async()                                  # block 0 (old generation) still in flight, never drained
    ctx.submit_host([blocks[1].ctypes.data], [len(blocks[1])], [2])
    ctx.wait_batch()
    old, new = Oracle(max_size=cmax), Oracle(max_size=cmax)
    compare_block(ctx.batch_result(0), old.reduce(blocks[0], 1), tag="old generation block")
    for _ in range(2):                                 # refused again while nothing was drained
        with pytest.raises(HdrfError) as ei:
            ctx.wait_batch()
        assert "drained" in str(ei.value), str(ei.value)
    disk = {}
    _apply(disk, ctx.drain_containers(buf_bytes=1 << 20))
    assert _check_files(disk, old, "old generation") > 0
    ctx.wait_batch()                                   # the same batch, now completed
    compare_block(ctx.batch_result(0), new.reduce(blocks[1], 2), tag="new generation block")
    compare_state(ctx, new, [2], tag="after the refused switch", containers=False)
    disk2 = {}
    _apply(disk2, ctx.drain_containers(buf_bytes=1 << 20))
    _check_files(disk2, new, "new generation")

    # forced: a view completes the switch batch anyway -> the old containers are dropped, the context is lost
    ctx.submit_host([blocks[2].ctypes.data], [len(blocks[2])], [3])     # generation 2, in flight, never drained
    ctx.reset_async()
    ctx.submit_host([blocks[3].ctypes.data], [len(blocks[3])], [4])     # generation 3
    with pytest.raises(HdrfError) as ei:
        ctx.index_count()
    assert "undrained" in str(ei.value), str(ei.value)
    ctx.reset()
    fresh = Oracle(max_size=cmax)
    ctx.submit_host([blocks[3].ctypes.data], [len(blocks[3])], [4])
    ctx.wait_batch()
    compare_block(ctx.batch_result(0), fresh.reduce(blocks[3], 4), tag="after hdrf_reset")
    ctx.close()


def test_reset_async_then_restore_then_submit():
    """A restore between hdrf_reset_async and the next submit (a DataNode re-initialised while blocks
    were in flight, then restarted from persisted Redis state and chunkDir files) is kept: the pending
    generation is applied before the restore, not after it.  The blocks after it equal an oracle that
    never stopped."""
    cmax = 1 << 20
    roots = corpus_roots(131, 500000, 9, 4)
    blocks = [corpus_block_host(131, roots, b, 4, 1 << 18) for b in range(9)]
    size = len(blocks[0])
    ids = [0x900 + b for b in range(9)]
    ctx = Context(container_max=cmax, max_block_bytes=1 << 20, max_batch_blocks=3, index_log2=18, arena_slots=64)
    dev = ctx.dev_alloc(size * 9 + 4096)
    ctx.h2d(dev, np.concatenate(blocks))
    total = size * 9 + 4096

    def batch(b0):
        return ([dev + (b0 + i) * size for i in range(3)], [size] * 3, [total - (b0 + i) * size for i in range(3)],
                ids[b0:b0 + 3])

    ctx.reduce_batch(*batch(0))
    keys, vals = ctx.index_dump()
    alloc = ctx.allocator()
    recipes = {i: ctx.recipe(i) for i in ids[:3]}
    opens = []
    for t in range(3):
        d, closed = ctx.container(int.from_bytes(alloc[3 * t:3 * t + 3], "big"))
        opens.append(d if d is not None and not closed else None)
    ctx.submit_batch(*batch(3))                        # in flight across the reset
    ctx.reset_async()
    ctx.wait_batch()
    ctx.index_load(keys, vals)                         # the restore: pending generation applied first
    ctx.allocator_load(alloc, opens)
    for i, r in recipes.items():
        ctx.recipe_load(i, r)
    ora = Oracle(max_size=cmax)
    for b in range(3):
        ora.reduce(blocks[b], ids[b])
    ctx.submit_batch(*batch(6))
    ctx.wait_batch()
    for i in range(3):
        compare_block(ctx.batch_result(i), ora.reduce(blocks[6 + i], ids[6 + i]), tag=f"after restore, block {i}")
    compare_state(ctx, ora, ids[:3] + ids[6:], tag="restore after reset_async", containers=False)
    ctx.dev_free(dev)
    ctx.close()
