"""hdrf_reset_async: a fresh DataNode from the next submit on, without draining the batches in flight
(the bench's back-to-back steps).  The batches submitted before it complete against the old state,
those after it against a fresh index, allocator, containers and recipes — each sequence equal to its
own oracle run, for compressor 1 and 2, across several resets (epochs) and a forced epoch wrap."""
import numpy as np
import pytest

from helpers import compare_block, compare_state
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
    order; a durable-container context refuses the asynchronous form."""
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
    d = Context(container_max=1 << 20, max_block_bytes=1 << 20, max_batch_blocks=2, index_log2=16, arena_slots=32,
                retain_containers=1)
    with pytest.raises(HdrfError):
        d.reset_async()
    d.close()
