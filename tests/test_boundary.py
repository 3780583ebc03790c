"""The drop-in boundary's contract: concurrent callers with
arrival tickets, and durable containers handed out as chunkDir file operations.

- Tickets: DataXceiver threads take a ticket when their block arrives and reduce later from their
  own thread in any order; the result is the reference's FIFO order (AIWriteQueue,
  DN/DataDeduplicator.java:124-158; DN/DDRunner.java:20-36).
- Durable containers (cfg.retain_containers): every closed container and every open-container
  append is drained as the file operation the storer performs on chunkDir + id
  (DN/DataDeduplicator.java:748-818); the files equal the oracle's containers, the arena ring wraps
  without losing anything, a submit that could overwrite an undrained container is refused, and
  every block rebuilds from the drained files alone.
"""
import threading

import numpy as np
import pytest

from helpers import compare_block, compare_state, make_block, prng_bytes
from hdrf_amd.lib import Context, HdrfError
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu


def _blocks(seed, n, size, dup_div=3):
    """n blocks: two pieces of size // dup_div from a shared base (cross-block duplicates) + new random bytes."""
    rng = np.random.default_rng(seed)
    base = [make_block(k, seed + i, 600_000) for i, k in enumerate(["random", "text", "binary"])]
    out = []
    d = size // dup_div
    for i in range(n):
        parts = [base[int(rng.integers(3))][int(rng.integers(0, 200_000)):][:d] for _ in range(2)]
        out.append(np.concatenate(parts + [make_block("random", seed + 100 + i, size - 2 * d)]))
    return out


def test_ticketed_threads_reduce_in_arrival_order():
    """One thread per block (the DDRunner shape, DN/BlockReceiver.java:1261), tickets taken in
    arrival order, threads started in REVERSE order so later blocks reach the native call first:
    every result and the final index / containers / recipes / allocator equal the sequential
    oracle run in ticket (arrival) order."""
    import time
    blocks = _blocks(31, 6, 700_000)
    ids = [4000 + i for i in range(6)]
    ctx = Context(container_max=1 << 20, max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=20, arena_slots=64)
    tickets = [ctx.ticket_take() for _ in blocks]          # arrival order 0..5
    assert tickets == sorted(tickets)
    results, errors = {}, []

    def worker(b):
        try:
            results[b] = ctx.reduce_block(blocks[b], ids[b], ticket=tickets[b])
        except Exception as e:                             # noqa: BLE001 - surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(b,)) for b in range(6)]
    for b in reversed(range(6)):
        th[b].start()
        time.sleep(0.05)
    for t in th:
        t.join(60)
    assert not any(t.is_alive() for t in th), "ticketed reductions did not finish"
    assert not errors, errors
    ora = Oracle(max_size=1 << 20)
    for b in range(6):
        compare_block(results[b], ora.reduce(blocks[b], ids[b]), tag=f"ticket {b}")
    compare_state(ctx, ora, ids, tag="tickets")
    # a cancelled ticket does not hold up the ones after it
    t0, t1 = ctx.ticket_take(), ctx.ticket_take()
    ctx.ticket_cancel(t0)
    extra = make_block("random", 77, 50_000)
    compare_block(ctx.reduce_block(extra, 4100, ticket=t1), ora.reduce(extra, 4100), tag="after cancel")
    ctx.close()


def test_threads_with_racing_views_are_serialised():
    """Threads taking tickets as their blocks "arrive" (order recorded), reducing with them and
    reading views (index count) while the other threads reduce: the state is the oracle's for the
    recorded arrival order, so the context lock serialised every call."""
    blocks = _blocks(41, 6, 300_000)
    ids = [5000 + i for i in range(6)]
    ctx = Context(container_max=1 << 20, max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=20, arena_slots=64)
    order, lock, errors = [], threading.Lock(), []

    def worker(t):
        try:
            for b in (t, t + 3):
                tk = None
                with lock:                                   # arrival = this thread's turn at the lock
                    tk = ctx.ticket_take()
                    order.append(b)
                ctx.reduce_block(blocks[b], ids[b], ticket=tk)
                ctx.index_count()                            # a view racing the other threads' reductions
        except Exception as e:                               # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors
    ora = Oracle(max_size=1 << 20)
    for b in order:
        ora.reduce(blocks[b], ids[b])
    compare_state(ctx, ora, ids, tag="serialised")
    ctx.close()


def _apply(disk, events):
    """The storer's file operations on a dict chunkDir: closed -> rewrite, open -> write at offset."""
    for cid, closed, off, data in events:
        if off == 0:                                  # (re)write: a new file, or a closed Lz4Codec file
            disk[cid] = (bytearray(data), bool(closed))
        else:                                         # the file grows (closed: its last bytes, compressor 1)
            f = disk.get(cid, (bytearray(), False))[0]
            assert len(f) == off, f"append to {cid} at {off}, file has {len(f)}"
            f[off:] = data
            disk[cid] = (f, bool(closed))


@pytest.mark.parametrize("compressor", [1, 2])
def test_durable_containers_drain_wrap_and_rebuild(compressor):
    cmax = 1 << 20
    blocks = _blocks(51 + compressor, 22, 2 << 20, dup_div=8)   # ~1.5 MiB new per block: the 8-slot rings wrap
    ids = [6000 + i for i in range(len(blocks))]
    kw = dict(compressor=compressor, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=20,
              arena_slots=32, retain_containers=1)
    # without drains the ring fills: the submit is refused BEFORE anything changes
    ctx0 = Context(**kw)
    with pytest.raises(HdrfError) as ei:
        for b, i in zip(blocks, ids):
            ctx0.reduce_block(b, i)
    assert ei.value.code == -4 and "drain" in str(ei.value)
    ctx0.close()

    ctx = Context(**kw)
    ora = Oracle(compressor=compressor, max_size=cmax)
    disk = {}
    for b, i in zip(blocks, ids):
        compare_block(ctx.reduce_block(b, i), ora.reduce(b, i), tag=f"durable block {i}")
        _apply(disk, ctx.drain_containers(buf_bytes=1 << 20))     # small buffer: several drain calls
    assert ctx.drain_containers() == []
    # the files are the oracle's containers, byte for byte (closed: raw or Lz4Codec; open: raw)
    alloc = ora.allocator()
    n_cont = 0
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, oc = ora.container(cid)
            if od is None:
                continue
            n_cont += 1
            assert cid in disk, f"container {cid} never drained"
            assert bytes(disk[cid][0]) == bytes(od) and disk[cid][1] == oc, f"container {cid} file differs"
    assert n_cont == len(disk) and n_cont > 8 * 3, "the ring of 8 slots per range must have wrapped"
    wrapped = sum(ctx.container(cid)[0] is None for cid in disk)
    assert wrapped > 0
    compare_state(ctx, ora, ids, tag=f"durable c{compressor}", containers=False)   # files compared above
    # a restarted DataNode with nothing but the Redis state and the drained files rebuilds every block
    keys, vals = ctx.index_dump()
    recipes = {i: ctx.recipe(i) for i in ids}
    ctx.close()
    ctx2 = Context(**kw)
    ctx2.index_load(keys, vals)
    for i, r in recipes.items():
        ctx2.recipe_load(i, r)
    for cid, (data, closed) in disk.items():
        ctx2.container_load(cid, bytes(data), closed and compressor == 2)
    for b, i in zip(blocks, ids):
        assert np.array_equal(ctx2.reconstruct_block(i), b), f"block {i} not rebuilt from drained files"
    ctx2.close()


@pytest.mark.parametrize("compressor", [1, 2])
def test_durable_drain_with_batches_in_flight(compressor):
    """The streaming DataNode shape (BASELINE config 5, hdrf_jni.c): blocks submitted from host
    memory three deep, and after every hdrf_wait_batch a drain hands out what the completed batches
    produced while the later ones keep running.  Every drained file equals the oracle's container
    (DN/DataDeduplicator.java:748-818) and nothing is lost when the rings wrap."""
    cmax = 1 << 20
    blocks = _blocks(71 + compressor, 40, 2 << 20, dup_div=8)
    ids = [6500 + i for i in range(len(blocks))]
    ctx = Context(compressor=compressor, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=1,
                  index_log2=20, arena_slots=64, retain_containers=1)
    ora = Oracle(compressor=compressor, max_size=cmax)
    disk, pend = {}, []
    for b, i in zip(blocks, ids):
        ctx.submit_host([b.ctypes.data], [len(b)], [i])
        pend.append((b, i))
        if len(pend) == 3:
            ctx.wait_batch()
            ob, oi = pend.pop(0)
            compare_block(ctx.batch_result(0), ora.reduce(ob, oi), tag=f"in-flight drain block {oi}")
            _apply(disk, ctx.drain_containers(buf_bytes=1 << 20))
    while pend:
        ctx.wait_batch()
        ob, oi = pend.pop(0)
        compare_block(ctx.batch_result(0), ora.reduce(ob, oi), tag=f"in-flight drain block {oi}")
        _apply(disk, ctx.drain_containers(buf_bytes=1 << 20))
    assert ctx.drain_containers() == []
    alloc = ora.allocator()
    n_cont = 0
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, oc = ora.container(cid)
            if od is None:
                continue
            n_cont += 1
            assert cid in disk and bytes(disk[cid][0]) == bytes(od) and disk[cid][1] == oc, f"container {cid}"
    assert n_cont == len(disk) and n_cont > 16 * 3, "the ring of 16 slots per range must have wrapped"
    assert sum(ctx.container(cid)[0] is None for cid in disk) > 0
    compare_state(ctx, ora, ids, tag=f"in-flight drain c{compressor}", containers=False)
    ctx.close()


def test_capacity_refusal_names_its_recovery():
    """a durable-container submit refused because the batches IN FLIGHT bound the ring
    (their closes cannot be drained yet) names hdrf_wait_batch; the documented recovery (wait the
    oldest, drain, submit again) succeeds.  With nothing in flight, undrained containers alone name
    hdrf_drain_containers.  Every block still equals the oracle's, every drained file its container."""
    cmax = 1 << 20
    blocks = _blocks(81, 10, 2 << 20, dup_div=8)
    ids = [6800 + i for i in range(len(blocks))]
    ctx = Context(container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=20, arena_slots=32,
                  retain_containers=1)
    ora = Oracle(max_size=cmax)
    disk, pend, refused_inflight = {}, [], 0

    def complete():
        ctx.wait_batch()
        ob, oi = pend.pop(0)
        compare_block(ctx.batch_result(0), ora.reduce(ob, oi), tag=f"recovery block {oi}")

    for b, i in zip(blocks, ids):
        try:
            ctx.submit_host([b.ctypes.data], [len(b)], [i])
        except HdrfError as e:
            assert e.code == -4 and "hdrf_wait_batch" in str(e), str(e)
            refused_inflight += 1
            complete()                                       # the oldest batch, then its containers
            _apply(disk, ctx.drain_containers())
            ctx.submit_host([b.ctypes.data], [len(b)], [i])  # the retry succeeds
        pend.append((b, i))
    assert refused_inflight > 0, "the ring never filled with a batch in flight"
    while pend:
        complete()
    # nothing in flight, nothing drained: the refusal names the drain
    extra = _blocks(82, 24, 2 << 20, dup_div=8)
    with pytest.raises(HdrfError) as ei:
        for j, b in enumerate(extra):
            ctx.reduce_block(b, 6900 + j)
            ora.reduce(b, 6900 + j)
    assert ei.value.code == -4 and "hdrf_drain_containers first" in str(ei.value), str(ei.value)
    _apply(disk, ctx.drain_containers())
    alloc = ora.allocator()
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, oc = ora.container(cid)
            if od is not None and cid in disk:
                assert bytes(disk[cid][0]) == bytes(od), f"container {cid}"
    ctx.close()


def test_pipeline_depth_is_refused_not_waited():
    """A submit beyond HDRF_PIPELINE_DEPTH returns HDRF_E_CAPACITY (the caller's awaitOldest pairs
    one to one with its submits) and leaves the batches in flight untouched."""
    from hdrf_amd.lib import PIPELINE_DEPTH as D
    blocks = _blocks(61, D + 1, 200_000)
    ctx = Context(container_max=1 << 20, max_block_bytes=1 << 20, max_batch_blocks=1, index_log2=18, arena_slots=16)
    ora = Oracle(max_size=1 << 20)
    for i in range(D):
        ctx.submit_host([blocks[i].ctypes.data], [len(blocks[i])], [7000 + i])
    with pytest.raises(HdrfError) as ei:
        ctx.submit_host([blocks[D].ctypes.data], [len(blocks[D])], [7000 + D])
    assert ei.value.code == -4
    for i in range(D):
        ctx.wait_batch()
        compare_block(ctx.batch_result(0), ora.reduce(blocks[i], 7000 + i), tag=f"depth {i}")
    with pytest.raises(HdrfError):
        ctx.wait_batch()                                     # nothing left in flight
    ctx.close()


def test_packet_receive_matches_oracle():
    """hdrf_rx_begin / hdrf_append_packet / hdrf_submit_slot (DN/BlockReceiver.java:877-896): blocks
    arrive as ragged packets, two blocks' packets interleaved, packet buffers overwritten right
    after each call; every block is reduced exactly like the sequential oracle in submit order."""
    rng = np.random.default_rng(71)
    blocks = _blocks(71, 6, 900_000)
    blocks[2] = blocks[2][:3]                                  # a 3-byte block
    blocks[4] = np.zeros(0, np.uint8)                          # an empty block
    ids = [8000 + i for i in range(len(blocks))]
    ctx = Context(container_max=1 << 20, max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=20, arena_slots=64)
    ora = Oracle(max_size=1 << 20)
    scratch = np.zeros(1 << 21, np.uint8)                      # the "network buffer", reused per packet

    def packets(b):
        o, out = 0, []
        while o < len(b):
            n = int(rng.choice([1, 700, 65536, 100_003, 1 << 20]))
            out.append(b[o:o + n])
            o += n
        return out

    pending = []
    order = []
    for pair in ((0, 1), (2, 3), (4, 5)):
        rxs = {b: ctx.rx_begin(ids[b]) for b in pair}
        queues = {b: packets(blocks[b]) for b in pair}
        while any(queues.values()):                            # interleave the two blocks' packets
            for b in pair:
                if queues[b]:
                    p = queues[b].pop(0)
                    scratch[:len(p)] = p
                    ctx.append_packet(rxs[b], scratch.ctypes.data, len(p))
                    scratch[:len(p)] = 0xA5                    # the caller reuses its buffer at once
        for b in pair:
            if len(pending) == 3:
                ctx.wait_batch()
                g = pending.pop(0)
                compare_block(ctx.batch_result(0), ora.reduce(blocks[g], ids[g]), tag=f"packet block {g}")
            ctx.submit_slot(rxs[b])
            pending.append(b)
            order.append(b)
    while pending:
        ctx.wait_batch()
        g = pending.pop(0)
        compare_block(ctx.batch_result(0), ora.reduce(blocks[g], ids[g]), tag=f"packet block {g}")
    compare_state(ctx, ora, ids, tag="packets")
    ctx.close()


def test_packet_rounds_submitted_as_batches():
    """hdrf_submit_slots (JNI submitBlocks): the blocks received in one round go in as ONE batch in
    the order listed (the FIFO), a round of 1, 3 and 4 blocks including an empty one; the per-block
    results and the final state equal the sequential oracle's.  A repeated or unknown receive
    buffer, or more blocks than max_batch_blocks, is refused before anything is submitted, and the
    buffers are free again once the batch completes."""
    rng = np.random.default_rng(73)
    blocks = _blocks(73, 8, 700_000)
    blocks[5] = np.zeros(0, np.uint8)
    ids = [8600 + i for i in range(len(blocks))]
    ctx = Context(container_max=1 << 20, max_block_bytes=2 << 20, max_batch_blocks=4, index_log2=20, arena_slots=64)
    ora = Oracle(max_size=1 << 20)
    rounds = [[0], [1, 2, 3], [4, 5, 6, 7]]
    pending = []
    for rnd in rounds:
        rxs = [ctx.rx_begin(ids[b]) for b in rnd]
        for b, rx in zip(rnd, rxs):
            o = 0
            while o < len(blocks[b]):
                n = int(rng.choice([1000, 65536, 300_001]))
                p = np.ascontiguousarray(blocks[b][o:o + n])
                ctx.append_packet(rx, p.ctypes.data, len(p))
                o += n
        if len(rxs) > 1:
            with pytest.raises(HdrfError) as ei:                  # the same buffer twice
                ctx.submit_slots([rxs[0], rxs[0]])
            assert ei.value.code == -1
        with pytest.raises(HdrfError) as ei:                      # more than max_batch_blocks
            ctx.submit_slots(rxs + [rxs[0]] * (5 - len(rxs)))
        assert ei.value.code == -1
        ctx.submit_slots(rxs)
        pending.append(rnd)
        if len(pending) == 2:
            ctx.wait_batch()
            done = pending.pop(0)
            assert ctx.last_nblocks() == len(done)
            for i, b in enumerate(done):
                compare_block(ctx.batch_result(i), ora.reduce(blocks[b], ids[b]), tag=f"round block {b}")
    while pending:
        ctx.wait_batch()
        done = pending.pop(0)
        assert ctx.last_nblocks() == len(done)
        for i, b in enumerate(done):
            compare_block(ctx.batch_result(i), ora.reduce(blocks[b], ids[b]), tag=f"round block {b}")
    with pytest.raises(HdrfError):                                # no such receive buffer any more
        ctx.submit_slots([0])
    rxs = [ctx.rx_begin(9000 + k) for k in range(16)]             # all sixteen are free again
    for rx in rxs:
        ctx.rx_cancel(rx)
    compare_state(ctx, ora, ids, tag="packet rounds")
    ctx.close()


def test_packet_receivers_on_concurrent_threads():
    """Four receiver threads (one per block, as DataXceiver threads are) append their blocks' ragged
    packets at the same time (hdrf_append_packet takes no context lock); the blocks are then
    submitted in arrival order and every one matches the sequential oracle."""
    import threading
    blocks = _blocks(93, 4, 3_000_000)
    ids = [9100 + i for i in range(len(blocks))]
    ctx = Context(container_max=1 << 20, max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=20, arena_slots=64)
    ora = Oracle(max_size=1 << 20)
    rxs = [ctx.rx_begin(i) for i in ids]
    errs = []

    def receive(b):
        try:
            rng = np.random.default_rng(200 + b)
            buf = np.zeros(1 << 20, np.uint8)                  # this receiver's packet buffer, reused
            o = 0
            while o < len(blocks[b]):
                n = int(rng.choice([1, 513, 65536, 200_001, 1 << 20]))
                p = blocks[b][o:o + n]
                buf[:len(p)] = p
                ctx.append_packet(rxs[b], buf.ctypes.data, len(p))
                buf[:len(p)] = 0x5A
                o += len(p)
        except Exception as e:                                  # noqa: BLE001 (reported below)
            errs.append(e)

    th = [threading.Thread(target=receive, args=(b,)) for b in range(len(blocks))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    for b in range(len(blocks)):
        ctx.submit_slot(rxs[b])
        ctx.wait_batch()
        compare_block(ctx.batch_result(0), ora.reduce(blocks[b], ids[b]), tag=f"threaded packets {b}")
    compare_state(ctx, ora, ids, tag="threaded packets")
    ctx.close()


def test_packet_receivers_race_submit_and_wait():
    """Receivers keep appending on their threads while the main thread submits and waits on the
    blocks that finished earlier (hdrf_append_packet without the lock beside hdrf_submit_slot /
    hdrf_wait_batch under it); every block matches the sequential oracle."""
    import threading
    blocks = _blocks(95, 6, 2_500_000)
    ids = [9300 + i for i in range(len(blocks))]
    ctx = Context(container_max=1 << 20, max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=20, arena_slots=64)
    ora = Oracle(max_size=1 << 20)
    rxs = [ctx.rx_begin(i) for i in ids]
    errs = []

    def receive(b):
        try:
            rng = np.random.default_rng(300 + b)
            buf = np.zeros(1 << 20, np.uint8)
            o = 0
            while o < len(blocks[b]):
                n = int(rng.choice([1, 4096, 65536, 300_001]))
                p = blocks[b][o:o + n]
                buf[:len(p)] = p
                ctx.append_packet(rxs[b], buf.ctypes.data, len(p))
                o += len(p)
        except Exception as e:                                  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=receive, args=(b,)) for b in range(len(blocks))]
    for t in th:
        t.start()
    pending = []
    for b in range(len(blocks)):                               # arrival order; later receivers still run
        th[b].join()
        assert not errs, errs
        ctx.submit_slot(rxs[b])
        pending.append(b)
        if len(pending) == 2:
            ctx.wait_batch()
            g = pending.pop(0)
            compare_block(ctx.batch_result(0), ora.reduce(blocks[g], ids[g]), tag=f"race block {g}")
    while pending:
        ctx.wait_batch()
        g = pending.pop(0)
        compare_block(ctx.batch_result(0), ora.reduce(blocks[g], ids[g]), tag=f"race block {g}")
    compare_state(ctx, ora, ids, tag="race packets")
    ctx.close()


def test_packet_receive_cancel_overflow_and_reset_guard():
    """hdrf_rx_cancel gives back an abandoned receive buffer (more than the 16 buffers are abandoned,
    some with staging chunks still copying); a packet that would pass max_block_bytes -- including a
    length that wraps a 64-bit sum -- is refused without copying; hdrf_reset refuses while a block is
    being received.  A block received afterwards reduces exactly."""
    ctx = Context(container_max=1 << 20, max_block_bytes=12 << 20, max_batch_blocks=1, index_log2=20, arena_slots=64)
    ora = Oracle(max_size=1 << 20)
    junk = prng_bytes(5, 9 << 20)
    for k in range(19):                                        # > 16 abandoned receives
        rx = ctx.rx_begin(7000 + k)
        n = (k % 11 + 1) * (800 << 10)                         # up to 8.6 MiB: staging chunks flushed
        ctx.append_packet(rx, junk.ctypes.data, n)
        if k == 0:
            with pytest.raises(HdrfError):
                ctx.reset()                                    # a block is being received
            with pytest.raises(HdrfError):
                ctx.append_packet(rx, junk.ctypes.data, (1 << 64) - 1)    # r.len + len wraps
            with pytest.raises(HdrfError):
                ctx.append_packet(rx, junk.ctypes.data, (12 << 20) - n + 1)
        ctx.rx_cancel(rx)
        with pytest.raises(HdrfError):
            ctx.rx_cancel(rx)                                  # not receiving any more
    ctx.reset()
    blk = _blocks(97, 1, 3_000_000)[0]
    rx = ctx.rx_begin(7100)
    for o in range(0, len(blk), 65536):
        p = np.ascontiguousarray(blk[o:o + 65536])
        ctx.append_packet(rx, p.ctypes.data, len(p))
    ctx.submit_slot(rx)
    ctx.wait_batch()
    compare_block(ctx.batch_result(0), ora.reduce(blk, 7100), tag="after cancels")
    compare_state(ctx, ora, [7100], tag="after cancels")
    ctx.close()
