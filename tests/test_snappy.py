"""Stream-mode Snappy oracle (compressor == 0, DN/BlockReceiver.java:826-873,887-894,1238-1256):
google/snappy's raw compressor restated in oracle/hdrf_oracle.c and Hadoop SnappyCodec's
BlockCompressorStream framing (256 KiB buffer, MAX_INPUT 218,422).  Hadoop's libsnappy is not in
this image, so parity vs Hadoop is UNPINNED; the restatement is pinned byte for byte against the
snappy bundled in pyarrow (committed fixtures, tests/golden/make_snappy_fixtures.py, plus a live
comparison when pyarrow is importable) and by round trips through pyarrow's decoder."""
import os

import numpy as np
import pytest

from helpers import make_block
from oracle.oracle import hadoop_stream, hadoop_stream_decode, snappy_raw, snappy_raw_decode

KINDS = ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"]
SNAPPY_MAX_IN = 218_422
PKT = 64_512

try:
    import pyarrow as pa
    HAVE_PA = pa.Codec.is_available("snappy")
except Exception:  # pragma: no cover - pyarrow is part of this image
    HAVE_PA = False


def test_golden_fixtures_match_pyarrow_snappy():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "snappy_pyarrow.npz"))
    for i, (kind, n) in enumerate(zip(z["kinds"], z["sizes"])):
        d = make_block(str(kind), 1000 + i, int(n)).tobytes()
        assert snappy_raw(d) == z[f"out{i}"].tobytes(), f"fixture {i} ({kind}, {n})"


@pytest.mark.skipif(not HAVE_PA, reason="pyarrow snappy not importable")
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", [0, 1, 15, 16, 17, 100, 4096, 65_535, 65_536, 65_537, 200_000])
def test_raw_matches_pyarrow(kind, n):
    d = make_block(kind, n * 7 + 1, n).tobytes()
    c = snappy_raw(d)
    assert c == pa.compress(d, codec="snappy", asbytes=True)
    assert snappy_raw_decode(c, n) == d


def _elements(c):
    """Walk a raw snappy buffer: (varint length, [(kind, len, offset)])."""
    i = sh = raw = 0
    while True:
        b = c[i]; i += 1
        raw |= (b & 0x7F) << sh; sh += 7
        if not b & 0x80:
            break
    out = []
    while i < len(c):
        t = c[i]; i += 1
        if t & 3 == 0:
            ln = (t >> 2) + 1
            if ln > 60:
                k = ln - 60
                ln = int.from_bytes(c[i:i + k], "little") + 1
                i += k
            out.append(("lit", ln, 0)); i += ln
        elif t & 3 == 1:
            out.append(("c1", 4 + ((t >> 2) & 7), ((t >> 5) << 8) | c[i])); i += 1
        elif t & 3 == 2:
            out.append(("c2", (t >> 2) + 1, int.from_bytes(c[i:i + 2], "little"))); i += 2
        else:
            out.append(("c4", (t >> 2) + 1, int.from_bytes(c[i:i + 4], "little"))); i += 4
    return raw, out


@pytest.mark.parametrize("kind", ["text", "lowent", "zeros", "periodic"])
def test_format_invariants(kind):
    """Copies never cross a 64 KiB fragment (fresh table per fragment), use the 1-byte-offset
    form exactly when len < 12 and offset < 2048, and never exceed 64 bytes."""
    n = 300_000
    d = make_block(kind, 5, n).tobytes()
    raw, els = _elements(snappy_raw(d))
    assert raw == n
    pos = 0
    for k, ln, off in els:
        if k != "lit":
            assert 4 <= ln <= 64 and off <= pos % 65536
            assert (k == "c1") == (ln < 12 and off < 2048)
            assert k != "c4"
        pos += ln
    assert pos == n


def test_decoder_rejects_malformed():
    d = make_block("text", 3, 10_000).tobytes()
    c = snappy_raw(d)
    assert snappy_raw_decode(c[:-3], len(d)) is None               # truncated
    assert snappy_raw_decode(b"\x05\x01\x00", 5) is None           # copy before any output
    assert snappy_raw_decode(b"\x0a\x0c" + b"abcd", 10) is None     # short of the declared length


@pytest.mark.parametrize("n", [0, 1, 100, SNAPPY_MAX_IN, SNAPPY_MAX_IN + 1, 600_000])
def test_stream_single_write_is_one_framing(n):
    """One write() of the block: groups of MAX_INPUT bytes under one BE32 length when the write
    is larger than MAX_INPUT (then close() adds BE32 0), else one [raw][clen][snappy] group."""
    d = make_block("text", n + 3, n).tobytes()
    f = hadoop_stream(0, d, [n] if n else [])
    assert hadoop_stream_decode(0, f, n) == d
    if n == 0:
        assert f == b"\0\0\0\0"
    elif n <= SNAPPY_MAX_IN:
        c = int.from_bytes(f[4:8], "big")
        assert f[:4] == n.to_bytes(4, "big") and f[8:] == snappy_raw(d) and c == len(f) - 8
    else:
        assert f[:4] == n.to_bytes(4, "big") and f.endswith(b"\0\0\0\0")
        i, o = 4, 0
        while o < n:
            c = int.from_bytes(f[i:i + 4], "big")
            m = min(SNAPPY_MAX_IN, n - o)
            assert f[i + 4:i + 4 + c] == snappy_raw(d[o:o + m])
            i += 4 + c
            o += m


@pytest.mark.parametrize("kind", ["random", "text", "lowent"])
def test_stream_packets(kind):
    """Packet writes: groups of whole packets up to MAX_INPUT (3 x 64,512 B), no trailer."""
    n = 1_000_000
    d = make_block(kind, 9, n).tobytes()
    writes = [PKT] * (n // PKT) + ([n % PKT] if n % PKT else [])
    f = hadoop_stream(0, d, writes)
    assert hadoop_stream_decode(0, f, n) == d
    per = SNAPPY_MAX_IN // PKT
    i = o = 0
    while i < len(f):
        raw = int.from_bytes(f[i:i + 4], "big")
        c = int.from_bytes(f[i + 4:i + 8], "big")
        assert raw == min(per * PKT, n - o)
        blk = f[i + 8:i + 8 + c]
        assert blk == snappy_raw(d[o:o + raw])
        if HAVE_PA:
            assert pa.decompress(blk, raw, codec="snappy", asbytes=True) == d[o:o + raw]
        i += 8 + c
        o += raw
    assert o == n


def test_stream_ragged_writes():
    d = make_block("lowent", 4, 700_000).tobytes()
    f = hadoop_stream(0, d, [1000, 0, 50_000, 400_000, 249_000])
    assert hadoop_stream_decode(0, f, len(d)) == d
    assert f[:4] == (51_000).to_bytes(4, "big")
    f2 = hadoop_stream(0, d, [1000, 699_000])
    assert f2.endswith(b"\0\0\0\0") and hadoop_stream_decode(0, f2, len(d)) == d


def test_stream_codec4_is_the_lz4_stream():
    from oracle.oracle import hadoop_lz4_stream
    d = make_block("text", 2, 300_000).tobytes()
    w = [PKT] * 4 + [300_000 - 4 * PKT]
    assert hadoop_stream(4, d, w) == hadoop_lz4_stream(d, w)


def _varint(b, p):
    v = s = 0
    while True:
        c = b[p]
        p += 1
        v |= (c & 0x7F) << s
        s += 7
        if c < 0x80:
            return v, p


@pytest.mark.gpu
@pytest.mark.skipif(not HAVE_PA, reason="pyarrow snappy not present")
def test_gpu_snappycodec_files_decode_through_pyarrow_snappy():
    """The product's SnappyCodec files (the GPU stream pass, no oracle in between) decode group by
    group, block by block, through pyarrow's libsnappy to the input, for packet-sized and single writes."""
    from hdrf_amd.lib import Context
    ctx = Context(max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=16, arena_slots=16)
    kinds = ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"]
    d = np.concatenate([make_block(k, 300 + i, 150_001) for i, k in enumerate(kinds)])
    for writes in ([d.size], [64_512] * (d.size // 64_512) + [d.size % 64_512], [1000, 0, 250_000, d.size - 251_000]):
        f = ctx.stream_block_host(0, 81, d, writes)
        out, p = [], 0
        while p < len(f):
            ulen = int.from_bytes(f[p:p + 4], "big")
            p += 4
            got = 0
            while got < ulen:
                clen = int.from_bytes(f[p:p + 4], "big")
                blk = f[p + 4:p + 4 + clen]
                n, _ = _varint(blk, 0)
                out.append(pa.decompress(blk, decompressed_size=n, codec="snappy", asbytes=True))
                p += 4 + clen
                got += n
        assert b"".join(out) == d.tobytes(), writes
    ctx.close()
