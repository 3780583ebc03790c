"""GPU parity: the HIP path (libhdrf.so through its C-ABI) against the CPU oracle on the same
inputs, bit-exact: chunk boundaries, digests, dedup decisions, storeSize, container placement
and bytes, the final index (every digest -> 11-byte value), allocator and recipes."""
import numpy as np
import pytest

from helpers import compare_block, compare_state, make_block, prng_bytes
from hdrf_amd.corpus import corpus_block_host, corpus_roots
from hdrf_amd.lib import Context, HdrfError
from oracle.oracle import Oracle, chunk as ora_chunk, java_random_bytes

pytestmark = pytest.mark.gpu

SMALL = dict(max_block_bytes=16 << 20, max_batch_blocks=8, index_log2=20, arena_slots=64)


def run_sequence(blocks, hasher=0, container_max=1 << 25, compressor=1, **cfg):
    kw = dict(SMALL)
    kw.update(cfg)
    ctx = Context(hasher=hasher, container_max=container_max, compressor=compressor, **kw)
    ora = Oracle(hasher=hasher, compressor=compressor, max_size=container_max)
    ids = []
    for i, blk in enumerate(blocks):
        bid = 0x1000 + 7 * i
        g = ctx.reduce_block(blk, bid)
        o = ora.reduce(blk, bid)
        compare_block(g, o, tag=f"block {i}")
        ids.append(bid)
    compare_state(ctx, ora, ids)
    ctx.close()


@pytest.mark.parametrize("kind", ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"])
def test_chunking_kinds(kind):
    blk = make_block(kind, 17, 3 * 1024 * 1024 + 123)
    run_sequence([blk], segment_bytes=1 << 16)


@pytest.mark.parametrize("n", [0, 1, 15, 16, 700, 701, 702, 703, 1403, 1404, 1500, 4095, 65536 + 7])
def test_tiny_and_edge_sizes(n):
    run_sequence([make_block("random", n + 3, n), make_block("random", n + 3, n)])


def test_many_segments_random_large():
    blk = make_block("random", 99, 9 * 1024 * 1024 + 5)
    for seg in (1 << 16, 1 << 20):
        run_sequence([blk], segment_bytes=seg)


@pytest.mark.parametrize("kind", ["periodic", "zeros", "text", "sparse"])
def test_more_boundaries_than_stitch_nodes(kind):
    """A 132 MiB block at 64 KiB segments has 2112 segment boundaries, more than the 1,024 irregular
    boundaries one LDS window of the stitch holds (chunk.hip kStitchNodes): the windowed stitch
    compacts the ordered node list window by window and follows any number of them (round 3), and a
    path that ends at an unrepaired boundary continues with the sequential walk; the cuts are the
    oracle's either way."""
    blk = make_block(kind, 23, 132 * 1024 * 1024 + 77)
    run_sequence([blk], segment_bytes=1 << 16, max_block_bytes=136 << 20, max_batch_blocks=1)


@pytest.mark.parametrize("hasher", [0, 1])
def test_long_chunk_sha_lanes(hasher):
    """Chunks >= 64 KiB (the config-4 corpus's text segments hold forced 1,000,000-B cuts) are
    hashed on sha_full's dedicated long lanes once a completed batch has shown them (sha.hip): the
    first blocks run without them, the later ones with them, all bit-exact."""
    roots = corpus_roots(3, 0, 1, 24)
    mixed = corpus_block_host(3, roots, 0, 24, 1 << 20, mixed=True)
    r = make_block("random", 2, 700_000)
    blocks = [r, mixed[: 12 << 20], np.concatenate([r, mixed[5 << 20:]]), mixed[::-1].copy(), mixed]
    run_sequence(blocks, hasher=hasher, max_block_bytes=32 << 20)


def test_cross_block_dups_and_intra_block_dups():
    a = make_block("random", 1, 600_000)
    b = make_block("random", 2, 400_000)
    blocks = [a, np.concatenate([a[:300_000], b]), np.concatenate([b, b]), a, make_block("text", 3, 250_000),
              np.zeros(0, np.uint8), a[:5000]]
    run_sequence(blocks)


@pytest.mark.parametrize("hasher", [0, 1])
def test_container_flushes_small_containers(hasher):
    # 2^20-byte containers force closes; 3 ranges per block
    roots = corpus_roots(5, 300000, 6, 8)
    blocks = [corpus_block_host(5, roots, b, 8, 1 << 18) for b in range(6)]
    run_sequence(blocks, hasher=hasher, container_max=1 << 20)


def test_java_random_block_config1():
    # BASELINE config 1: one block of java.util.Random(seed).nextBytes in 1024-B pieces
    # (DFSTestUtil.createFile); 16 MiB here, the 128 MiB case is test_config1_full_block.
    blk = java_random_bytes(0xDEADBEEF, 1024, 16 << 20)
    run_sequence([blk])


def test_batch_api_matches_sequential_oracle():
    roots = corpus_roots(9, 500000, 12, 8)
    blocks = [corpus_block_host(9, roots, b, 8, 1 << 19) for b in range(12)]
    ctx = Context(**SMALL)
    ora = Oracle()
    size = len(blocks[0])
    dev = ctx.dev_alloc(size * len(blocks) + 4096)
    ctx.h2d(dev, np.concatenate(blocks))
    total = size * len(blocks) + 4096
    ids = []
    for start in range(0, 12, 5):                        # batches of 5, 5, 2
        nb = min(5, 12 - start)
        ptrs = [dev + (start + i) * size for i in range(nb)]
        lens = [size] * nb
        readable = [total - (start + i) * size for i in range(nb)]
        bids = [500 + start + i for i in range(nb)]
        ctx.reduce_batch(ptrs, lens, readable, bids)
        for i in range(nb):
            g = ctx.batch_result(i)
            o = ora.reduce(blocks[start + i], bids[i])
            compare_block(g, o, tag=f"batch block {start + i}")
        ids += bids
    compare_state(ctx, ora, ids)
    ctx.dev_free(dev)
    ctx.close()


def test_batch_with_mixed_kinds_and_sizes():
    kinds = ["random", "periodic", "zeros", "text", "random", "sparse", "ff", "random"]
    blocks = [make_block(k, 40 + i, 1_500_000 + 7777 * i) for i, k in enumerate(kinds)]
    blocks[4] = blocks[0].copy()                          # whole-block duplicate in the same batch
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


def test_config1_full_block_boundaries():
    # full 128 MiB java.util.Random block: boundaries + digests + decisions bit-exact
    blk = java_random_bytes(0x5EED, 1024, 128 << 20)
    ctx = Context(max_block_bytes=128 << 20, max_batch_blocks=1, index_log2=20, arena_slots=16)
    ora = Oracle()
    g = ctx.reduce_block(blk, 1)
    o = ora.reduce(blk, 1)
    compare_block(g, o, "config1")
    # property at full size: re-reducing the same block is all-duplicate, stores nothing
    g2 = ctx.reduce_block(blk, 2)
    assert not g2["is_new"].any() and g2["store_size"] == 0
    ctx.close()


def test_errors_fail_loudly():
    ctx = Context(**SMALL)
    with pytest.raises(HdrfError):
        ctx.reduce_block(np.zeros((16 << 20) + 1, np.uint8), 1)      # larger than max_block_bytes
    with pytest.raises(HdrfError):
        ctx.reduce_batch([0x1001], [10], [10], [1])                   # unaligned, no slack
    ctx.close()


@pytest.mark.parametrize("bits", [16, 20])
def test_index_tag_collisions_take_exact_slow_path(bits):
    # test hook: index tags truncated to `bits` bits, so distinct digests collide on the tag and
    # must be told apart by the stored digest bytes (apply verify + single-thread slow path)
    roots = corpus_roots(21, 400000, 8, 8)
    blocks = [corpus_block_host(21, roots, b, 8, 1 << 19) for b in range(8)]
    run_sequence(blocks, debug_tag_bits=bits)
    # batched too (collisions between blocks of one batch)
    ctx = Context(debug_tag_bits=bits, **SMALL)
    ora = Oracle()
    size = len(blocks[0])
    dev = ctx.dev_alloc(size * 8 + 4096)
    ctx.h2d(dev, np.concatenate(blocks))
    ctx.reduce_batch([dev + i * size for i in range(8)], [size] * 8, [size * (8 - i) + 4096 for i in range(8)],
                     list(range(40, 48)))
    for i in range(8):
        compare_block(ctx.batch_result(i), ora.reduce(blocks[i], 40 + i), tag=f"coll batch {i}")
    compare_state(ctx, ora, list(range(40, 48)))
    ctx.dev_free(dev)
    ctx.close()


@pytest.mark.parametrize("hasher", [0, 1])
def test_compression_stage_lz4_containers(hasher):
    """compressor == 2: every closed container is the Lz4Codec file of its bytes
    (DN/DataDeduplicator.java:770-779), byte-identical to the oracle's lz4 r123 + Hadoop framing."""
    rng = np.random.default_rng(5 + hasher)
    kinds = ["random", "lowent", "text", "binary", "sparse", "random", "lowent", "binary"]
    blocks = []
    for i, k in enumerate(kinds):
        b = make_block(k, 40 + i, 900_000 + int(rng.integers(0, 100_000)))
        if i >= 4:                                     # cross-block duplicates
            b = np.concatenate([blocks[i - 4][:300_000], b[:600_000]])
        blocks.append(b)
    run_sequence(blocks, hasher=hasher, container_max=1 << 20, compressor=2)


def test_compression_stage_large_container():
    """32 MiB containers (129 LZ4 segments each, close() trailer) on mixed data."""
    blocks = [np.concatenate([make_block(k, 70 + i, 6 << 20) for k in ("lowent", "random", "binary")])
              for i in range(3)]
    run_sequence(blocks, compressor=2, max_block_bytes=32 << 20, arena_slots=16)


@pytest.mark.parametrize("mixed", [False, True])
def test_device_corpus_matches_host_and_reduces(mixed):
    """hdrf_corpus_fill(_kind) == hdrf_amd.corpus.corpus_block_host byte for byte (configs 2 and 4),
    and the config-4 batch path (dedup + Lz4Codec containers) matches the oracle."""
    nb, spb, seg = 10, 8, 1 << 18
    roots = corpus_roots(33, 500000, nb, spb)
    ctx = Context(compressor=2 if mixed else 1, container_max=1 << 20, **SMALL)
    size = spb * seg
    dev = ctx.dev_alloc(size * nb + 4096)
    ctx.corpus_fill(dev, roots, nb, spb, seg, 33, mixed=mixed)
    blocks = [corpus_block_host(33, roots, b, spb, seg, mixed=mixed) for b in range(nb)]
    for b in range(nb):
        assert np.array_equal(ctx.d2h(dev + b * size, size), blocks[b]), f"corpus block {b}"
    ora = Oracle(compressor=2 if mixed else 1, max_size=1 << 20)
    ids = list(range(700, 700 + nb))
    for start in range(0, nb, 4):
        k = min(4, nb - start)
        ctx.reduce_batch([dev + (start + i) * size for i in range(k)], [size] * k,
                         [size * (nb - start - i) + 4096 for i in range(k)], ids[start:start + k])
        for i in range(k):
            compare_block(ctx.batch_result(i), ora.reduce(blocks[start + i], ids[start + i]), tag=f"block {start + i}")
    compare_state(ctx, ora, ids)
    st = ctx.stats()
    assert st["blocks"] == nb and st["logical_bytes"] == nb * size
    if mixed:
        assert st["closed_containers"] > 0 and st["closed_file_bytes"] < st["closed_raw_bytes"]
    ctx.dev_free(dev)
    ctx.close()


def test_pipelined_submit_wait_matches_sequential_oracle():
    """hdrf_submit_batch / hdrf_wait_batch: up to PIPELINE_DEPTH batches in flight (chunking, SHA
    and index/store on three streams) give the same results as the sequential oracle; a submit
    beyond the depth is refused with HDRF_E_CAPACITY (every submit pairs with one wait) and changes
    nothing."""
    from hdrf_amd.lib import PIPELINE_DEPTH as D
    nb, spb, seg = 14, 8, 1 << 18
    roots = corpus_roots(77, 500000, nb, spb)
    blocks = [corpus_block_host(77, roots, b, spb, seg) for b in range(nb)]
    ctx = Context(container_max=1 << 20, **SMALL)
    ora = Oracle(max_size=1 << 20)
    size = spb * seg
    dev = ctx.dev_alloc(size * nb + 4096)
    ctx.h2d(dev, np.concatenate(blocks))
    groups = [list(range(s, min(s + 2, nb))) for s in range(0, nb, 2)]
    ids = [900 + b for b in range(nb)]

    def check(group):
        assert ctx.last_nblocks() == len(group)
        for i, b in enumerate(group):
            compare_block(ctx.batch_result(i), ora.reduce(blocks[b], ids[b]), tag=f"pipelined block {b}")

    pending = []
    for gi, g in enumerate(groups):
        args = ([dev + b * size for b in g], [size] * len(g), [size * (nb - b) + 4096 for b in g], [ids[b] for b in g])
        if len(pending) == D:                # pipeline full: refused, the caller waits first
            with pytest.raises(HdrfError) as ei:
                ctx.submit_batch(*args)
            assert ei.value.code == -4
            ctx.wait_batch()
            check(pending.pop(0))
        ctx.submit_batch(*args)
        pending.append(g)
        if gi % 4 != 3:                      # mostly keep the pipeline full
            continue
        while len(pending) > 1:
            ctx.wait_batch()
            check(pending.pop(0))
    while pending:
        ctx.wait_batch()
        check(pending.pop(0))
    compare_state(ctx, ora, ids)
    ctx.dev_free(dev)
    ctx.close()


@pytest.mark.parametrize("hasher,compressor", [(0, 1), (1, 1), (0, 2)])
def test_reconstruct_round_trip(hasher, compressor):
    """Read side (DataConstructor, DN/DataConstructor.java:73-250,360-531): every reduced block is
    rebuilt from its recipe, the index and the containers, byte for byte; closed Lz4Codec container
    files decode (oracle framing decoder) to the raw container the gather reads."""
    from oracle.oracle import hadoop_lz4_decode
    rng = np.random.default_rng(11 + hasher)
    base = [make_block(k, 60 + i, 700_000) for i, k in enumerate(["random", "lowent", "text", "binary"])]
    blocks = []
    for i in range(9):
        parts = [base[int(rng.integers(4))][int(rng.integers(0, 300_000)):][:200_000] for _ in range(3)]
        blocks.append(np.concatenate(parts + [make_block("random", 90 + i, 150_000)]))
    blocks += [np.zeros(0, np.uint8), make_block("random", 5, 1000), blocks[2]]
    ctx = Context(hasher=hasher, compressor=compressor, container_max=1 << 20, **SMALL)
    ora = Oracle(hasher=hasher, compressor=compressor, max_size=1 << 20)
    for i, b in enumerate(blocks):
        ctx.reduce_block(b, 300 + i)
        ora.reduce(b, 300 + i)
    for i, b in enumerate(blocks):
        assert np.array_equal(ctx.reconstruct_block(300 + i), b), f"block {i} not rebuilt"
    if compressor == 2:
        alloc = ctx.allocator()
        n = 0
        for t in range(3):
            last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
            for cid in range(t << 22, last):
                data, closed = ctx.container(cid)
                od, _ = ora.container(cid)
                if data is None or not closed:
                    continue
                assert data == od, f"container {cid:#x} file differs"
                raw = hadoop_lz4_decode(data, 1 << 21)
                assert raw is not None and 0 < len(raw) <= (1 << 20)
                n += 1
        assert n > 0
    ctx.close()


@pytest.mark.parametrize("compressor", [1, 2])
def test_scheme_plugin_round_trip(compressor):
    """The Python mirror of the plugin API (hdrf_amd/scheme.py): reduce -> length -> reconstruct
    in DataNode order, against the oracle's recipes."""
    from hdrf_amd.scheme import HipReductionScheme
    blocks = [make_block("random", 400, 900_000), make_block("text", 401, 600_000)]
    blocks.append(np.concatenate([blocks[0][:300_000], blocks[1]]))
    sch = HipReductionScheme(hasher=0, compressor=compressor, container_max=1 << 20, **SMALL)
    ora = Oracle(hasher=0, compressor=compressor, max_size=1 << 20)
    for i, b in enumerate(blocks):
        sch.reduce(b, 700 + i)
        ora.reduce(b, 700 + i)
    for i, b in enumerate(blocks):
        assert sch.length(700 + i) == len(b)
        assert sch.recipe(700 + i) == ora.recipe(700 + i)
        assert sch.reconstruct(700 + i) == b.tobytes()
    with pytest.raises(HdrfError):
        sch.reconstruct(12345)
    sch.close()


def test_submit_host_streaming_matches_sequential_oracle():
    """The streaming write path (hdrf_submit_host, BASELINE config 5): host-resident blocks of
    ragged lengths, pinned and pageable, copied H2D on the side stream while earlier batches are
    reduced, give exactly the sequential oracle's results and state."""
    from hdrf_amd.lib import PIPELINE_DEPTH as D
    rng = np.random.default_rng(5)
    base = [make_block(k, 70 + i, 600_000) for i, k in enumerate(["random", "text", "lowent", "binary"])]
    blocks = []
    for i in range(15):
        n = [0, 1, 700, 701, 4097, 333_333, 1_000_003][i % 7]
        parts = [base[int(rng.integers(4))][int(rng.integers(0, 200_000)):][:n // 2],
                 make_block("random", 500 + i, n - n // 2)]
        blocks.append(np.concatenate(parts)[:n])
    ctx = Context(container_max=1 << 20, **SMALL)
    ora = Oracle(max_size=1 << 20)
    pinned = ctx.host_alloc(sum(len(b) for b in blocks) + 1)
    ptrs, o = [], 0
    for i, b in enumerate(blocks):
        if i % 2:                                   # odd blocks from pinned memory, odd offsets
            pinned[o:o + len(b)] = b
            ptrs.append(pinned.ctypes.data + o)
            o += len(b) + 1
        else:
            ptrs.append(b.ctypes.data if len(b) else 0)
    ids = [1000 + i for i in range(len(blocks))]
    groups = [list(range(s, min(s + 4, len(blocks)))) for s in range(0, len(blocks), 4)]
    pending = []

    def check(g):
        for i, b in enumerate(g):
            compare_block(ctx.batch_result(i), ora.reduce(blocks[b], ids[b]), tag=f"host block {b}")

    for g in groups:
        if len(pending) == D:
            ctx.wait_batch()
            check(pending.pop(0))
        ctx.submit_host([ptrs[b] for b in g], [len(blocks[b]) for b in g], [ids[b] for b in g])
        pending.append(g)
    while pending:
        ctx.wait_batch()
        check(pending.pop(0))
    compare_state(ctx, ora, ids)
    for i, b in enumerate(blocks):
        assert np.array_equal(ctx.reconstruct_block(ids[i]), b)
    ctx.host_free(pinned)
    ctx.close()


@pytest.mark.parametrize("case", ["packets", "ragged", "single", "empty", "tail_large"])
def test_stream_mode_lz4_file_matches_oracle(case):
    """Stream-mode scheme compressor 4 (DN/BlockReceiver.java:846-855,887-894,1238-1256): the GPU
    writes the oracle's Lz4Codec file byte for byte for every write pattern, and records the
    block length."""
    from oracle.oracle import hadoop_lz4_stream
    n = {"packets": 3_000_000, "ragged": 1_200_000, "single": 700_000, "empty": 0, "tail_large": 900_000}[case]
    parts = [make_block(k, 80 + i, n // 4 + 1) for i, k in enumerate(["text", "random", "binary", "zeros"])]
    d = np.concatenate(parts)[:n]
    writes = {"packets": [64_512] * (n // 64_512) + [n % 64_512],
              "ragged": [1000, 0, 50_000, 600_000, 249_000, 300_000], "single": [n], "empty": [],
              "tail_large": [1000, 899_000]}[case]
    ctx = Context(**SMALL)
    dev = ctx.dev_alloc(n + 4096)
    if n:
        ctx.h2d(dev, d)
    f = ctx.stream_block(4, 77, dev, n, n + 4096, writes)
    assert f == hadoop_lz4_stream(d, writes)
    assert ctx.block_length(77) == n
    from oracle.oracle import lzop_stream
    assert ctx.stream_block(3, 78, dev, n, n + 4096, writes) == bytes(lzop_stream(d, writes))   # LzopCodec
    with pytest.raises(HdrfError):
        ctx.stream_block(7, 79, dev, n, n + 4096, writes)          # no such codec
    ctx.dev_free(dev)
    ctx.close()


@pytest.mark.parametrize("kind", ["random", "text", "zeros", "lowent", "binary", "periodic"])
def test_lz4_file_decode_round_trip(kind):
    """GPU Lz4Codec decoder (read side, DN/DataConstructor.java:171-176,495-500): the oracle's
    container framing and stream-mode framing (packet writes, a large write) decode to the raw
    bytes; a corrupted file is rejected."""
    from oracle.oracle import hadoop_lz4, hadoop_lz4_stream
    n = 1_300_000
    d = make_block(kind, 31, n).tobytes()
    ctx = Context(**SMALL)
    for f in (hadoop_lz4(d), hadoop_lz4(d[:5000]), hadoop_lz4(b""),
              hadoop_lz4_stream(d, [64_512] * (n // 64_512) + [n % 64_512]),
              hadoop_lz4_stream(d, [1000, 700_000, n - 701_000])):
        out = ctx.lz4_file_decode(f, n)
        assert out == d[:len(out)] and len(out) in (0, 5000, n)
    good = hadoop_lz4(d)
    for bad in (good[:-1],                            # truncated
                good[:4] + (int.from_bytes(good[4:8], "big") - 1).to_bytes(4, "big") + good[8:-1],   # short block
                good[:4] + b"\x7f\xff\xff\xff" + good[8:]):      # block length past the end
        with pytest.raises(HdrfError):
            ctx.lz4_file_decode(bad, n)
    ctx.close()


@pytest.mark.parametrize("case", ["packets", "ragged", "single", "empty", "tail_large", "kinds"])
def test_stream_mode_snappy_file_matches_oracle(case):
    """Stream-mode scheme compressor 0 (SnappyCodec, DN/BlockReceiver.java:826-873,887-894): the
    GPU writes the oracle's SnappyCodec file byte for byte (MAX_INPUT 218,422 groups of
    independent 64 KiB snappy fragments) for every write pattern; codecs 3/5 stay unsupported."""
    from oracle.oracle import hadoop_stream
    n = {"packets": 3_000_000, "ragged": 1_200_000, "single": 700_000, "empty": 0, "tail_large": 900_000,
         "kinds": 8 * 70_001}[case]
    kinds = ["text", "random", "binary", "zeros"] if case != "kinds" else \
        ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"]
    parts = [make_block(k, 90 + i, n // len(kinds) + 1) for i, k in enumerate(kinds)]
    d = np.concatenate(parts)[:n]
    writes = {"packets": [64_512] * (n // 64_512) + [n % 64_512],
              "ragged": [1000, 0, 50_000, 600_000, 249_000, 300_000], "single": [n], "empty": [],
              "tail_large": [1000, 899_000], "kinds": [70_001] * 8}[case]
    ctx = Context(**SMALL)
    dev = ctx.dev_alloc(n + 4096)
    if n:
        ctx.h2d(dev, d)
    f = ctx.stream_block(0, 79, dev, n, n + 4096, writes)
    assert f == hadoop_stream(0, d, writes)
    assert ctx.stream_block_host(0, 80, d, writes) == f
    assert ctx.block_length(79) == n
    assert ctx.stream_file_decode(0, f, n) == d.tobytes()
    for codec in (1, 7):                                          # not stream codecs
        with pytest.raises(HdrfError):
            ctx.stream_block(codec, 78, dev, n, n + 4096, writes)
    ctx.dev_free(dev)
    ctx.close()


@pytest.mark.parametrize("kind", ["random", "text", "zeros", "lowent", "periodic", "sparse"])
def test_snappy_file_decode_round_trip(kind):
    """GPU SnappyCodec decoder (DataConstructor's compression-only read, DN/DataConstructor.java:
    102-220): oracle files of several write patterns decode to the raw bytes; corrupt files are
    rejected."""
    from oracle.oracle import hadoop_stream
    n = 1_100_000
    d = make_block(kind, 33, n).tobytes()
    ctx = Context(**SMALL)
    for w in ([n], [64_512] * (n // 64_512) + [n % 64_512], [1000, 700_000, n - 701_000]):
        assert ctx.stream_file_decode(0, hadoop_stream(0, d, w), n) == d
    assert ctx.stream_file_decode(0, hadoop_stream(0, d[:5000], [5000]), n) == d[:5000]
    assert ctx.stream_file_decode(0, hadoop_stream(0, b"", []), n) == b""
    good = hadoop_stream(0, d[:100_000], [100_000])
    for bad in (good[:-1],
                good[:4] + (int.from_bytes(good[4:8], "big") - 1).to_bytes(4, "big") + good[8:-1],
                good[:8] + b"\x00" + good[9:]):                     # varint length 0 != raw length
        with pytest.raises(HdrfError):
            ctx.stream_file_decode(0, bad, n)
    ctx.close()


def test_reconstruct_from_loaded_container_files():
    """A context whose arena slots were reused (small arena) cannot rebuild early blocks from
    device memory; after loading the chunkDir files of the missing containers (closed ones as
    Lz4Codec files, decoded on the GPU) every block reconstructs byte for byte."""
    cmax = 1 << 20
    blocks = [make_block(["random", "text", "binary"][i % 3], 600 + i, 900_000) for i in range(14)]
    ctx = Context(compressor=2, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=2, index_log2=20,
                  arena_slots=12)
    ora = Oracle(compressor=2, max_size=cmax)
    for i, b in enumerate(blocks):
        ctx.reduce_block(b, 40 + i)
        ora.reduce(b, 40 + i)
    missing = []
    for i, b in enumerate(blocks):
        try:
            assert np.array_equal(ctx.reconstruct_block(40 + i), b)
        except HdrfError:
            missing.append(i)
    assert missing, "the small arena should have evicted early containers"
    alloc = ora.allocator()
    loaded = 0
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            data, closed = ora.container(cid)
            if data is None:
                continue
            gd, _ = ctx.container(cid)
            if gd is None:                              # not resident any more: load its file
                ctx.container_load(cid, data, closed)
                loaded += 1
    assert loaded > 0
    for i in missing:
        assert np.array_equal(ctx.reconstruct_block(40 + i), blocks[i]), f"block {i}"
    ctx.close()


@pytest.mark.parametrize("hasher,compressor", [(0, 1), (1, 2)])
def test_restart_from_persisted_state(hasher, compressor):
    """Index persistence: a second context restored from the first one's Redis
    state (index rows, "blockID" allocator, recipes) and the open containers' chunkDir files
    continues exactly like a DataNode that never stopped: later blocks dedup against the restored
    index, append to the reopened containers, and every value, container, recipe and the
    allocator match the sequential oracle; old blocks reconstruct once their files are loaded."""
    cmax = 1 << 20
    rng = np.random.default_rng(3)
    base = [make_block(k, 90 + i, 800_000) for i, k in enumerate(["random", "text", "binary"])]
    blocks = []
    for i in range(14):
        parts = [base[int(rng.integers(3))][int(rng.integers(0, 300_000)):][:250_000] for _ in range(2)]
        blocks.append(np.concatenate(parts + [make_block("random", 700 + i, 300_000)]))
    ids = [2000 + i for i in range(len(blocks))]
    kw = dict(hasher=hasher, compressor=compressor, container_max=cmax, **SMALL)
    ctx1 = Context(**kw)
    ora = Oracle(hasher=hasher, compressor=compressor, max_size=cmax)
    for b, i in zip(blocks[:7], ids[:7]):
        ctx1.reduce_block(b, i)
        ora.reduce(b, i)
    keys, vals = ctx1.index_dump()
    alloc = ctx1.allocator()
    recipes = {i: ctx1.recipe(i) for i in ids[:7]}
    files = {}
    for t in range(3):
        for cid in range(t << 22, int.from_bytes(alloc[3 * t:3 * t + 3], "big") + 1):
            d, closed = ctx1.container(cid)
            if d is not None:
                files[cid] = (d, closed)
    opens = []
    for t in range(3):
        cid = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        d = files.get(cid)
        opens.append(d[0] if d is not None and not d[1] else None)
    ctx1.close()
    ctx2 = Context(**kw)                                 # the restarted DataNode
    ctx2.index_load(keys, vals)
    ctx2.allocator_load(alloc, opens)
    for i, r in recipes.items():
        ctx2.recipe_load(i, r)
    for b, i in zip(blocks[7:], ids[7:]):
        compare_block(ctx2.reduce_block(b, i), ora.reduce(b, i), tag=f"after restart, block {i}")
    gk, gv = ctx2.index_dump()
    ok, ov = ora.index_dump()
    assert np.array_equal(gk, ok) and np.array_equal(gv, ov)
    assert ctx2.allocator() == ora.allocator()
    for i in ids:
        assert ctx2.recipe(i) == ora.recipe(i)
    for cid, (d, closed) in files.items():               # chunkDir: closed files of the first run
        gd, _ = ctx2.container(cid)
        if gd is None:
            ctx2.container_load(cid, d, closed and compressor == 2)
    for i, b in zip(ids, blocks):
        assert np.array_equal(ctx2.reconstruct_block(i), b), f"block {i}"
    ctx2.close()


def test_probe_stats_count_every_chunk():
    """hdrf_probe_stats (steady-state index measurement) covers every chunk of the last batch; on a
    nearly full small table the probes get longer than on an empty one."""
    blocks = [make_block("random", 910 + i, 1_000_000) for i in range(4)]
    lens = []
    for log2 in (20, 13):
        ctx = Context(max_block_bytes=4 << 20, max_batch_blocks=4, index_log2=log2, arena_slots=16,
                      container_max=1 << 21)
        pinned = ctx.host_alloc(sum(len(b) for b in blocks))
        o, ptrs = 0, []
        for b in blocks:
            pinned[o:o + len(b)] = b
            ptrs.append(pinned.ctypes.data + o)
            o += len(b)
        ctx.submit_host(ptrs, [len(b) for b in blocks], [1, 2, 3, 4])
        ctx.wait_batch()
        n = sum(ctx.batch_info(i)[0] for i in range(4))
        s, m, c = ctx.probe_stats()
        assert c == n and m >= 0 and s >= 0
        lens.append(s / c)
        ctx.host_free(pinned)
        ctx.close()
    assert lens[1] > lens[0]


@pytest.mark.parametrize("hasher", [0, 1])
def test_reset_epochs_are_fresh_indexes(hasher):
    """hdrf_reset makes a fresh DataNode index by bumping the table's epoch (common.hpp: an entry
    tagged with an older epoch is empty) instead of clearing 2^k x 64 B.  The same blocks reduced
    again after a reset find their own previous-epoch entries at the very slots they probe (same
    digests, same tags); batched, the claims race those stale entries.  Every round equals a fresh
    oracle, index dump included — also after 300 resets (the 255-epoch wrap clears the table), and
    an index restored into a reset context (hdrf_index_load) is live and decides the next block."""
    roots = corpus_roots(33, 500000, 6, 4)
    blocks = [corpus_block_host(33, roots, b, 4, 1 << 20) for b in range(6)]
    size = len(blocks[0])
    ctx = Context(hasher=hasher, container_max=1 << 22, **SMALL)
    dev = ctx.dev_alloc(size * 6 + 4096)
    ctx.h2d(dev, np.concatenate(blocks))
    ids = list(range(60, 66))

    def one_round(tag):
        ora = Oracle(hasher=hasher, max_size=1 << 22)
        ctx.reduce_batch([dev + i * size for i in range(3)], [size] * 3, [size * (6 - i) + 4096 for i in range(3)],
                         ids[:3])
        for i in range(3):
            compare_block(ctx.batch_result(i), ora.reduce(blocks[i], ids[i]), tag=f"{tag} batch0 block {i}")
        for i in range(3, 6):
            compare_block(ctx.reduce_block(blocks[i], ids[i]), ora.reduce(blocks[i], ids[i]), tag=f"{tag} block {i}")
        compare_state(ctx, ora, ids, tag=tag)
        return ora

    one_round("epoch 1")
    for r in range(2):
        ctx.reset()
        one_round(f"after reset {r + 1}")
    for _ in range(300):
        ctx.reset()
    ora = one_round("after 300 resets")
    keys, vals = ctx.index_dump()
    ctx.reset()
    assert ctx.index_count() == 0, "a reset index holds no entry"
    ctx.index_load(keys, vals)
    k2, v2 = ctx.index_dump()
    assert np.array_equal(k2, keys) and np.array_equal(v2, vals), "restored index differs"
    extra = make_block("random", 7, 300_000)
    extra = np.concatenate([blocks[2][:400_000], extra])
    g = ctx.reduce_block(extra, 99)
    o = ora.reduce(extra, 99)
    for f in ("offsets", "digests", "is_new"):
        assert np.array_equal(g[f], o[f]), f"restored index: {f} differs"
    assert g["store_size"] == o["store_size"]
    ctx.dev_free(dev)
    ctx.close()


@pytest.mark.parametrize("hasher", [0, 1])
def test_product_against_independent_restatements(hasher):
    """No C oracle in between: the GPU's chunk END offsets equal the literal Python closed form of
    DataDeduplicator.chunking (oracle/pyref.py chunking_closed_form, DN/DataDeduplicator.java:264-307)
    and every digest equals hashlib's SHA-1 / SHA-224 of the chunk's bytes (DN/utilities.java:98-137)."""
    import hashlib
    from oracle import pyref
    h = hashlib.sha1 if hasher == 0 else hashlib.sha224
    ctx = Context(hasher=hasher, segment_bytes=1 << 16, **SMALL)
    for i, kind in enumerate(["random", "text", "lowent", "binary", "sparse", "periodic", "zeros"]):
        blk = make_block(kind, 500 + i, 700_000 + 977 * i)
        g = ctx.reduce_block(blk, 7000 + i)
        raw = blk.tobytes()
        assert list(g["offsets"]) == pyref.chunking_closed_form(raw), kind
        starts = [0] + list(g["offsets"][:-1])
        for j, (a, b) in enumerate(zip(starts, g["offsets"])):
            assert bytes(g["digests"][j]) == h(raw[a:b]).digest(), (kind, j)
    ctx.close()


def test_dedup_semantics_against_python_transliteration():
    """The whole reduction with no C oracle in between: a sequence of blocks with cross-block and
    intra-block duplicates through the GPU and through oracle/pyref.py's literal Python DataDeduplicator
    (dict Redis, hashlib; DN/DataDeduplicator.java:108-217, chunkMeta.java:35-77): the same cuts,
    digests, dedup decisions and storeSize per block, then the same index (every key, 11-byte value),
    allocator ("blockID"), recipes and container bytes — with 1.1 MB containers so flushes happen."""
    from oracle import pyref
    cmax = 1_100_000
    ctx = Context(container_max=cmax, **SMALL)
    ref = pyref.PyRef(max_size=cmax)
    base = [make_block(k, 900 + i, 1_000_000 + 1311 * i) for i, k in enumerate(["random", "text", "binary", "lowent"])]
    blocks = [base[0], base[1], base[0].copy(), np.concatenate([base[2][:500_000], base[1][100_000:]]),
              np.concatenate([base[3], base[3]]), base[2], make_block("random", 950, 30_000)]
    ids = []
    for i, blk in enumerate(blocks):
        bid = 0x3100 + i
        g, r = ctx.reduce_block(blk, bid), ref.reduce(blk.tobytes(), bid)
        assert list(g["offsets"]) == r["offsets"], i
        assert [bytes(x) for x in g["digests"]] == r["digests"], i
        assert list(g["is_new"]) == r["is_new"], i
        assert g["store_size"] == r["store_size"], i
        ids.append(bid)
    keys, vals = ctx.index_dump()
    gidx = {bytes(k): bytes(v) for k, v in zip(keys, vals)}
    ridx = {k: v for k, v in ref.redis.items() if len(k) == 20}
    assert gidx == ridx
    assert ctx.allocator() == ref.redis[b"blockID"]
    for bid in ids:
        assert ctx.recipe(bid) == ref.redis[(bid & 0xFFFFFFFF).to_bytes(4, "big")], bid
    for cid, data in ref.files.items():
        got, closed = ctx.container(cid)
        assert got == bytes(data), cid
        assert closed == (cid in ref.closed), cid
    assert ref.closed                                  # (the sequence does close containers)
    ctx.close()
