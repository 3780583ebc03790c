"""The LZ4 block encoder pinned against a real liblz4 (CPU).

The compression stage restates lz4 r123 ``LZ4_compress`` (hadoop-common 3.1.0's native
Lz4Compressor, `DN/DataDeduplicator.java:770-779` via Lz4Codec); neither r123 nor Hadoop is in the
image.  pyarrow 25.0.0 bundles a modern liblz4 (>= 1.9) and the system has liblz4 1.9.3; both parse
identically to each other (checked on every input below) and differ from r123 in exactly
three rules (oracle/hdrf_oracle.c ``lz4_compress_rules``: the search's step schedule, the search's
last position, and the 5-byte hash of byU32 tables on 64-bit hosts).  Run under those three rules
the oracle's encoder must equal liblz4's ``LZ4_compress_default`` byte for byte — which pins
everything the two parses share: the table fill, catch-up, the test of the next position, the
token / length / offset coding and the last literals — and the r123 output itself must decode
through liblz4's decoder.  The GPU pass equals the r123-rule oracle byte for byte (tests/test_lz4*.py),
so this is the external pin of its bytes short of Hadoop itself."""
import ctypes

import numpy as np
import pytest

from helpers import make_block
from hdrf_amd.corpus import corpus_block_host, corpus_roots
from oracle.oracle import hadoop_lz4, lz4_block, lz4_block_modern

pa = pytest.importorskip("pyarrow")


def _system_liblz4():
    try:
        L = ctypes.CDLL("liblz4.so.1")
    except OSError:
        return None
    L.LZ4_compress_default.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    L.LZ4_compress_default.restype = ctypes.c_int
    L.LZ4_versionNumber.restype = ctypes.c_int
    return L


SYS = _system_liblz4()

KINDS = ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"]
# below / at / above LZ4_minLength (13), the byU16 -> byU32 switch (64 KiB + 11), one Hadoop segment
SIZES = [0, 1, 5, 12, 13, 14, 15, 20, 31, 64, 100, 1000, 4096, 20000, 65535, 65546, 65547, 65548,
         70000, 131072, 200000, 261100]


def liblz4(d):
    """pyarrow's bundled liblz4; the system's (1.9.3 here) must agree with it."""
    c = pa.compress(d, codec="lz4_raw", asbytes=True)
    if SYS is not None:
        out = ctypes.create_string_buffer(len(d) + len(d) // 255 + 16)
        n = SYS.LZ4_compress_default(d, out, len(d), len(out))
        assert out.raw[:n] == c, "the two liblz4 builds disagree"
    return c


def test_two_liblz4_builds_present():
    if SYS is None:
        pytest.skip("no system liblz4")
    assert SYS.LZ4_versionNumber() >= 10900


@pytest.mark.parametrize("kind", KINDS)
def test_modern_rules_equal_liblz4(kind):
    bad = []
    for n in SIZES:
        for seed in (7, 8, 9):
            d = make_block(kind, seed, n)
            if lz4_block_modern(d) != liblz4(d.tobytes()):
                bad.append((n, seed))
    assert not bad, f"{kind}: oracle (liblz4 rules) != liblz4 at (size, seed) {bad}"


def test_modern_rules_equal_liblz4_on_the_config4_corpus():
    """Every 261,100-B segment (and the short tail) of config 4's mixed-entropy corpus blocks: the
    segments the GPU pass compresses in the bench."""
    roots = corpus_roots(4, 500000, 2, 16)
    for b in range(2):
        blk = corpus_block_host(4, roots, b, 16, 1 << 19, mixed=True)
        for off in range(0, blk.size, 261100):
            seg = blk[off:off + 261100]
            assert lz4_block_modern(seg) == liblz4(seg.tobytes()), f"block {b} segment at {off}"


def test_modern_rules_equal_liblz4_on_structured_edges():
    """Long matches (length continuation bytes at 15 / 270 / 525 / 780), long literal runs, matches
    at the 65,535-B distance limit and just past it, and matches ending at matchlimit."""
    r = make_block("random", 3, 300000)
    cases = []
    for ml in (4, 18, 19, 270, 271, 524, 525, 779, 780, 5000):
        cases.append(np.concatenate([r[:100], r[:ml], r[1000:1400]]))
    for lit in (14, 15, 16, 269, 270, 271, 525, 70000):
        cases.append(np.concatenate([r[:50], r[5000:5000 + lit], r[:50], r[9000:9100]]))
    for dist in (65530, 65535, 65536, 65540):
        cases.append(np.concatenate([r[:32], r[100000:100000 + dist - 32], r[:32], r[200000:200040]]))
    for tail in (0, 4, 5, 6, 11, 12, 13):
        cases.append(np.concatenate([r[:40], r[:40 + tail]]))
    cases.append(np.resize(r[:7], 200000))
    for i, d in enumerate(cases):
        assert lz4_block_modern(d) == liblz4(d.tobytes()), f"case {i} ({d.size} B)"


@pytest.mark.parametrize("seed", range(6))
def test_modern_rules_equal_liblz4_random_shapes(seed):
    """Seeded random sizes and kind splices (no fixed shape list)."""
    rng = np.random.default_rng(1000 + seed)
    for _ in range(12):
        parts = []
        for _ in range(int(rng.integers(1, 5))):
            kind = KINDS[int(rng.integers(len(KINDS)))]
            parts.append(make_block(kind, int(rng.integers(1 << 20)), int(rng.integers(0, 90000))))
        d = np.concatenate(parts)[:261100]
        assert lz4_block_modern(d) == liblz4(d.tobytes()), f"{d.size} B"


def test_each_rule_is_needed():
    """The three rules are the whole difference, and each one shows: with any one of them left at
    r123's, some input differs from liblz4 (so the comparison above is not vacuous)."""
    probes = [make_block(k, s, n) for k in ("zeros", "text", "lowent") for s in (7, 8)
              for n in (13, 20000, 65535, 70000, 261100)]
    for rule in (1, 2, 4):
        differs = [d.size for d in probes if lz4_block_modern(d, 7 & ~rule) != liblz4(d.tobytes())]
        assert differs, f"rule {rule} never matters on the probes"
    assert all(lz4_block_modern(d, 7) == liblz4(d.tobytes()) for d in probes)


@pytest.mark.parametrize("kind", KINDS)
def test_r123_blocks_decode_through_liblz4(kind):
    """The product's rules (r123): every block decodes through liblz4's decoder to the input."""
    for n in SIZES:
        d = make_block(kind, 11, n)
        c = lz4_block(d)
        if n == 0:
            assert c == b"\x00"
            continue
        assert pa.decompress(c, decompressed_size=n, codec="lz4_raw", asbytes=True) == d.tobytes(), n


def test_hadoop_frames_decode_segment_by_segment_through_liblz4():
    """Lz4Codec container files (BlockCompressorStream framing around r123 blocks): each
    [BE32 clen] block decodes through liblz4 to its 261,100-B segment."""
    roots = corpus_roots(5, 0, 1, 16)
    blk = corpus_block_host(5, roots, 0, 16, 1 << 16, mixed=True)[: 600000 + 77]
    f = hadoop_lz4(blk)
    assert int.from_bytes(f[:4], "big") == blk.size
    p, off = 4, 0
    while off < blk.size:
        clen = int.from_bytes(f[p:p + 4], "big")
        seg = blk[off:off + 261100]
        assert pa.decompress(f[p + 4:p + 4 + clen], decompressed_size=seg.size, codec="lz4_raw",
                             asbytes=True) == seg.tobytes()
        p += 4 + clen
        off += seg.size
    assert f[p:] == b"\x00\x00\x00\x00"


def _decode_lz4codec(f):
    """An Lz4Codec (BlockCompressorStream) file decoded group by group, each block by liblz4."""
    out, p = [], 0
    while p < len(f):
        ulen = int.from_bytes(f[p:p + 4], "big")
        p += 4
        got = 0
        while got < ulen:
            clen = int.from_bytes(f[p:p + 4], "big")
            seg = min(261100, ulen - got)
            out.append(pa.decompress(f[p + 4:p + 4 + clen], decompressed_size=seg, codec="lz4_raw", asbytes=True))
            p += 4 + clen
            got += seg
    return b"".join(out)


@pytest.mark.gpu
def test_gpu_lz4codec_files_decode_through_liblz4():
    """The product's bytes themselves (the GPU Lz4Codec pass, no oracle in between) decode through
    liblz4 to the input: every data kind at the table-switch and segment sizes, and config-4 corpus
    blocks split into several 261,100-B segments."""
    from hdrf_amd.lib import Context
    ctx = Context(max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=16, arena_slots=16)
    cases = [make_block(k, 21 + n, n) for k in KINDS for n in (13, 4096, 65546, 65547, 261100, 600000)]
    roots = corpus_roots(6, 500000, 2, 8)
    cases += [corpus_block_host(6, roots, b, 8, 1 << 18, mixed=True) for b in range(2)]
    for i, d in enumerate(cases):
        f = ctx.stream_block_host(4, 1, d, [d.size])
        assert _decode_lz4codec(f) == d.tobytes(), f"case {i} ({d.size} B)"
    ctx.close()
