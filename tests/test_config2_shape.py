"""GPU parity at the headline's real shape (BASELINE config 2, the bench's exact pipeline).

bench.py reduces 128 MiB corpus blocks in batches of up to 32 on a context opened with
max_block_bytes = 128 MiB, max_batch_blocks = 32 and the default 1 MiB speculation segment,
two batches in flight (hdrf_submit_batch / hdrf_wait_batch).  Here a few such blocks go
through that same context and pipeline, and EVERYTHING is compared with the sequential
oracle (DataDeduplicator + Redis + chunkDir restated, oracle/hdrf_oracle.c): chunk END
offsets, digests, is_new, storeSize, container placement, the full index dump (digest ->
11-B chunkMeta value), every container's bytes, the "blockID" allocator and the recipes.

A full-size block in the forced-cut regime (0xFF bytes are signed -1, so with M = max(0, ...)
= 0 no byte qualifies and every chunk is cut at 1,000,001 B, DN/DataDeduplicator.java:288-294)
with random islands goes through the same context.
"""
import numpy as np
import pytest

from helpers import compare_block, compare_state, prng_bytes
from hdrf_amd.corpus import corpus_roots
from hdrf_amd.lib import Context
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

S = 128 << 20
SEG = 1 << 20


def forced_cut_block(seed):
    """0xFF-filled 128 MiB with 4 KiB random islands every 9 MiB (some chunks cut at an island
    byte, the rest forced at 1,000,001 B)."""
    blk = np.full(S, 0xFF, np.uint8)
    isl = prng_bytes(seed, 4096 * 15)
    for i, o in enumerate(range(3 << 20, S - 4096, 9 << 20)):
        blk[o:o + 4096] = isl[(i % 15) * 4096:(i % 15 + 1) * 4096]
    return blk


def test_config2_shape_pipelined_full_state():
    nb, spb, seed = 6, S // SEG, 20251015
    roots = corpus_roots(seed, 500000, nb, spb)
    ctx = Context(max_block_bytes=S, max_batch_blocks=32, segment_bytes=SEG, index_log2=23, arena_slots=64)
    ora = Oracle()
    total = (nb + 1) * S + 4096
    dev = ctx.dev_alloc(total)
    ctx.corpus_fill(dev, roots, nb, spb, SEG, seed)
    ff = forced_cut_block(7)
    ctx.h2d(dev + nb * S, ff)
    blocks = [ctx.d2h(dev + b * S, S) for b in range(nb)] + [ff]
    ids = [b for b in range(nb + 1)]
    groups = [[0, 1, 2], [3, 4], [5, 6]]          # depth 2: submit, submit, wait, submit, wait, wait

    def submit(g):
        ctx.submit_batch([dev + b * S for b in g], [S] * len(g), [total - b * S for b in g], [ids[b] for b in g])

    def check(g):
        assert ctx.last_nblocks() == len(g)
        for i, b in enumerate(g):
            compare_block(ctx.batch_result(i), ora.reduce(blocks[b], ids[b]), tag=f"config2 block {b}")

    submit(groups[0])
    submit(groups[1])
    ctx.wait_batch()
    check(groups[0])
    submit(groups[2])
    ctx.wait_batch()
    check(groups[1])
    ctx.wait_batch()
    check(groups[2])
    compare_state(ctx, ora, ids, tag="config2")
    # size-independent property: every block rebuilds byte for byte from recipe + index + arena
    for b in (0, nb - 1, nb):
        assert np.array_equal(ctx.reconstruct_block(ids[b]), blocks[b]), f"block {b} not rebuilt"
    ctx.dev_free(dev)
    ctx.close()


def test_forced_cut_block_alone_and_one_block_calls():
    """hdrf_reduce_block (the JNI shape: one 128 MiB block per call) on the forced-cut block and
    on an all-0xFF block: boundaries at every 1,000,001 B, bit-exact."""
    ctx = Context(max_block_bytes=S, max_batch_blocks=1, index_log2=21, arena_slots=16)
    ora = Oracle()
    for i, blk in enumerate((forced_cut_block(11), np.full(S, 0xFF, np.uint8))):
        compare_block(ctx.reduce_block(blk, 50 + i), ora.reduce(blk, 50 + i), tag=f"forced {i}")
    ctx.close()


def test_config4_mixed_corpus_full_blocks():
    """BASELINE config 4's mixed-entropy 128 MiB blocks (1 MiB random / text / binary segments;
    text chains meet rarely, so many speculative boundaries go through the repair pass and jump
    segments) through the same pipeline, dedup + Lz4Codec containers: the full state matches."""
    nb, spb, seed = 3, S // SEG, 4242
    roots = corpus_roots(seed, 500000, nb, spb)
    ctx = Context(max_block_bytes=S, max_batch_blocks=32, segment_bytes=SEG, index_log2=22, arena_slots=64,
                  compressor=2)
    ora = Oracle(compressor=2)
    total = nb * S + 4096
    dev = ctx.dev_alloc(total)
    ctx.corpus_fill(dev, roots, nb, spb, SEG, seed, mixed=True)
    blocks = [ctx.d2h(dev + b * S, S) for b in range(nb)]
    ids = [300 + b for b in range(nb)]
    ctx.submit_batch([dev + b * S for b in (0, 1)], [S] * 2, [total - b * S for b in (0, 1)], ids[:2])
    ctx.submit_batch([dev + 2 * S], [S], [total - 2 * S], ids[2:])
    ctx.wait_batch()
    for i in range(2):
        compare_block(ctx.batch_result(i), ora.reduce(blocks[i], ids[i]), tag=f"config4 block {i}")
    ctx.wait_batch()
    compare_block(ctx.batch_result(0), ora.reduce(blocks[2], ids[2]), tag="config4 block 2")
    compare_state(ctx, ora, ids, tag="config4")
    ctx.dev_free(dev)
    ctx.close()


@pytest.mark.parametrize("arena_slots", [16, 64])
def test_config4_lz4_passes_overlap_across_batches(arena_slots):
    """Compressor 2 with the LZ4 pass of each batch on its own stream (alternating by batch), three
    batches in flight: batch k+1's place kernel reopens arena slots while batch k's LZ4 pass may
    still read its closed containers.  With 16 slots (4 per storer ring) the ring can wrap within
    the batches in flight, so stream B waits for the older LZ4 passes; with 64 it cannot, and the
    passes run concurrently.  Every container file, index value and recipe matches the oracle."""
    nb, seg, seed = 9, 1 << 20, 99
    size = 4 << 20
    roots = corpus_roots(seed, 400000, nb, size // seg)
    cmax = 4 << 20
    ctx = Context(max_block_bytes=size, max_batch_blocks=1, index_log2=20, arena_slots=arena_slots,
                  container_max=cmax, compressor=2)
    ora = Oracle(compressor=2, max_size=cmax)
    total = nb * size + 4096
    dev = ctx.dev_alloc(total)
    ctx.corpus_fill(dev, roots, nb, size // seg, seg, seed, mixed=True)
    blocks = [ctx.d2h(dev + b * size, size) for b in range(nb)]
    ids = [900 + b for b in range(nb)]
    pend = []
    for b in range(nb):
        ctx.submit_batch([dev + b * size], [size], [total - b * size], [ids[b]])
        pend.append(b)
        if len(pend) == 3:
            ctx.wait_batch()
            d = pend.pop(0)
            compare_block(ctx.batch_result(0), ora.reduce(blocks[d], ids[d]), tag=f"lz4 overlap block {d}")
    while pend:
        ctx.wait_batch()
        d = pend.pop(0)
        compare_block(ctx.batch_result(0), ora.reduce(blocks[d], ids[d]), tag=f"lz4 overlap block {d}")
    st = ctx.stats()
    assert st["closed_containers"] >= 3
    compare_state(ctx, ora, ids, tag=f"lz4 overlap {arena_slots}")
    ctx.dev_free(dev)
    ctx.close()
