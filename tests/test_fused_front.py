"""GPU parity of the fused chunk + fingerprint front (HDRF_FUSED=1, hdrf_amd/csrc/lanehash.hip;
DESIGN.md §6b) against the CPU oracle: the same cuts, digests, decisions, containers and final
state as the two-pass front.  The front is chosen when a context opens, so these tests set the
variable around their own contexts only."""
import numpy as np
import pytest

from helpers import compare_block, compare_state, make_block
from hdrf_amd.corpus import corpus_block_host, corpus_roots
from hdrf_amd.lib import Context
from oracle.oracle import Oracle

pytestmark = pytest.mark.gpu

SMALL = dict(max_block_bytes=16 << 20, max_batch_blocks=8, index_log2=20, arena_slots=64)


@pytest.fixture
def fused(monkeypatch):
    monkeypatch.setenv("HDRF_FUSED", "1")


def run_sequence(blocks, hasher=0, container_max=1 << 25, compressor=1, **cfg):
    kw = dict(SMALL)
    kw.update(cfg)
    ctx = Context(hasher=hasher, container_max=container_max, compressor=compressor, **kw)
    ora = Oracle(hasher=hasher, compressor=compressor, max_size=container_max)
    ids = []
    for i, blk in enumerate(blocks):
        bid = 0x2000 + 5 * i
        compare_block(ctx.reduce_block(blk, bid), ora.reduce(blk, bid), tag=f"block {i}")
        ids.append(bid)
    compare_state(ctx, ora, ids)
    ctx.close()


@pytest.mark.parametrize("kind", ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"])
def test_fused_chunking_kinds(fused, kind):
    """Every data kind the two-pass tests use, at 64 KiB segments (many boundaries: synced ones take
    the boundary digest, repaired ones the listed fix-up)."""
    run_sequence([make_block(kind, 17, 3 * 1024 * 1024 + 123)], segment_bytes=1 << 16)


@pytest.mark.parametrize("n", [0, 1, 700, 701, 702, 703, 1403, 4095, 65536 + 7])
def test_fused_edge_sizes(fused, n):
    run_sequence([make_block("random", n + 3, n), make_block("random", n + 3, n)])


@pytest.mark.parametrize("hasher", [0, 1])
def test_fused_long_chunks_and_sha224(fused, hasher):
    """Forced 1,000,000-B cuts (the config-4 text segments) run past a lane's byte cap into the repair
    walk, which runs without granule maxima here; SHA-224 takes the same paths."""
    roots = corpus_roots(3, 0, 1, 24)
    mixed = corpus_block_host(3, roots, 0, 24, 1 << 20, mixed=True)
    r = make_block("random", 2, 700_000)
    run_sequence([r, mixed[: 12 << 20], np.concatenate([r, mixed[5 << 20:]])], hasher=hasher,
                 max_block_bytes=32 << 20)


def test_fused_batch_mixed_kinds(fused):
    """One batch of mixed kinds and sizes with an in-batch whole-block duplicate (the batch API)."""
    kinds = ["random", "periodic", "zeros", "text", "random", "sparse", "ff", "random"]
    blocks = [make_block(k, 40 + i, 1_500_000 + 7777 * i) for i, k in enumerate(kinds)]
    blocks[4] = blocks[0].copy()
    ctx = Context(segment_bytes=1 << 16, **SMALL)
    ora = Oracle()
    align = lambda x: (x + 4095) // 4096 * 4096  # noqa: E731
    offs = np.cumsum([0] + [align(len(b)) for b in blocks])
    buf = np.zeros(offs[-1] + 4096, np.uint8)
    for b, o in zip(blocks, offs):
        buf[o:o + len(b)] = b
    dev = ctx.dev_alloc(buf.size)
    ctx.h2d(dev, buf)
    ids = list(range(900, 900 + len(blocks)))
    ctx.reduce_batch([dev + int(o) for o in offs[:-1]], [len(b) for b in blocks],
                     [int(buf.size - o) for o in offs[:-1]], ids)
    for i, b in enumerate(blocks):
        compare_block(ctx.batch_result(i), ora.reduce(b, ids[i]), tag=f"{kinds[i]}#{i}")
    compare_state(ctx, ora, ids)
    ctx.dev_free(dev)
    ctx.close()


def test_fused_and_two_pass_contexts_side_by_side(monkeypatch):
    """The front is read per context: a fused and a two-pass context in one process give the same
    cuts and digests for the same corpus blocks."""
    roots = corpus_roots(9, 500000, 4, 8)
    blocks = [corpus_block_host(9, roots, b, 8, 1 << 19) for b in range(4)]
    monkeypatch.setenv("HDRF_FUSED", "1")
    a = Context(**SMALL)
    monkeypatch.setenv("HDRF_FUSED", "0")
    b = Context(**SMALL)
    for i, blk in enumerate(blocks):
        ga, gb = a.reduce_block(blk, 10 + i), b.reduce_block(blk, 10 + i)
        assert np.array_equal(ga["offsets"], gb["offsets"]) and np.array_equal(ga["digests"], gb["digests"])
        assert ga["store_size"] == gb["store_size"]
    a.close()
    b.close()
