"""Compression stage oracle (compressor == 2): lz4 r123 LZ4_compress + Hadoop Lz4Codec
BlockCompressorStream framing (DN/DataDeduplicator.java:770-779).  Hadoop 3.1.0's bundled lz4
is not in this image, so compressed-byte parity vs Hadoop is UNPINNED; these tests pin the
restatement by (1) exact round trips through liblz4 1.9.3's independent LZ4_decompress_safe,
(2) the framing's structure, (3) the LZ4 format invariants (last 5 bytes literals, offsets
<= 65535, no match starts in the last 12 bytes)."""
import ctypes
import ctypes.util

import numpy as np
import pytest

from helpers import make_block
from oracle.oracle import hadoop_lz4, hadoop_lz4_decode, lz4_block, lz4_block_decode

KINDS = ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"]
SIZES = [0, 1, 5, 12, 13, 14, 100, 4096, 65535, 65546, 65547, 65548, 200_000, 261_100]


def _liblz4():
    for name in ("liblz4.so.1", ctypes.util.find_library("lz4")):
        if not name:
            continue
        try:
            L = ctypes.CDLL(name)
            L.LZ4_decompress_safe.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
            L.LZ4_decompress_safe.restype = ctypes.c_int
            return L
        except OSError:
            continue
    return None


def _parse_sequences(blk):
    """Walk an LZ4 block: yields (literal_len, offset or None, match_len)."""
    i, out = 0, []
    while i < len(blk):
        tok = blk[i]; i += 1
        lit = tok >> 4
        if lit == 15:
            while True:
                b = blk[i]; i += 1; lit += b
                if b != 255:
                    break
        i += lit
        if i == len(blk):
            out.append((lit, None, 0))
            break
        off = blk[i] | (blk[i + 1] << 8); i += 2
        ml = tok & 15
        if ml == 15:
            while True:
                b = blk[i]; i += 1; ml += b
                if b != 255:
                    break
        out.append((lit, off, ml + 4))
    return out


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", SIZES)
def test_lz4_block_round_trip_liblz4(kind, n):
    data = make_block(kind, n + 11, n).tobytes()
    blk = lz4_block(data)
    assert len(blk) <= n + n // 255 + 16
    assert lz4_block_decode(blk, n) == data
    L = _liblz4()
    if L is None:
        pytest.skip("liblz4 not present")
    out = ctypes.create_string_buffer(max(n, 1))
    got = L.LZ4_decompress_safe(blk, out, len(blk), n)
    assert got == n and out.raw[:n] == data


@pytest.mark.parametrize("kind", ["random", "text", "zeros", "binary", "lowent"])
def test_lz4_format_invariants(kind):
    n = 150_000
    data = make_block(kind, 5, n).tobytes()
    seqs = _parse_sequences(lz4_block(data))
    pos = 0
    for lit, off, ml in seqs:
        pos += lit
        if off is None:
            break
        assert 1 <= off <= 65535
        assert pos <= n - 12, "a match starts inside the last MFLIMIT bytes"
        pos += ml
        assert pos <= n - 5, "a match covers the last LASTLITERALS bytes"
    assert pos == n
    if kind in ("zeros", "lowent", "binary"):
        assert len(seqs) > 1          # compressible data produces matches


def test_hadoop_framing_structure():
    for n in (0, 1, 1000, 261_100, 261_101, 522_200, 600_000, 3 * 1024 * 1024):
        data = make_block("text", n, n).tobytes()
        f = hadoop_lz4(data)
        assert int.from_bytes(f[:4], "big") == n
        if n == 0:
            assert f == b"\0\0\0\0"
            continue
        i, segs = 4, []
        while i < len(f):
            c = int.from_bytes(f[i:i + 4], "big")
            if c == 0:
                assert i + 4 == len(f) and n > 261_100       # close() trailer after segmented writes
                break
            segs.append(f[i + 4:i + 4 + c]); i += 4 + c
        assert len(segs) == (n + 261_099) // 261_100
        assert b"".join(lz4_block_decode(s, 261_100) for s in segs) == data
        assert hadoop_lz4_decode(f, n) == data
        if n <= 261_100:
            assert i == len(f)                                 # no trailer for a single segment


# ---- stream mode (compressor 4): Lz4Codec output stream fed one write() per packet ----------
PKT = 64_512          # HDFS packet payload: 126 chunks x 512 B (64 KiB packets incl. checksums)


@pytest.mark.parametrize("n", [0, 1, 100, 261_100, 261_101, 600_000])
def test_stream_single_write_equals_one_shot_frame(n):
    """One write() of the whole block is exactly the dedup-mode container framing."""
    from oracle.oracle import hadoop_lz4_stream
    d = make_block("text", n + 3, n).tobytes()
    assert hadoop_lz4_stream(d, [n] if n else []) == hadoop_lz4(d)


@pytest.mark.parametrize("kind", ["random", "text", "zeros", "binary"])
def test_stream_packets_structure_and_round_trip(kind):
    """Packet writes: groups of whole packets up to MAX_INPUT (261,100 B), each
    [BE32 raw][BE32 clen][block], no trailer; decodes (oracle + framing decoder) to the block."""
    from oracle.oracle import hadoop_lz4_stream
    n = 1_500_000
    d = make_block(kind, 9, n).tobytes()
    writes = [PKT] * (n // PKT) + ([n % PKT] if n % PKT else [])
    f = hadoop_lz4_stream(d, writes)
    assert hadoop_lz4_decode(f, n) == d
    per = 261_100 // PKT                          # whole packets per group (4)
    i = o = 0
    groups = 0
    while i < len(f):
        raw = int.from_bytes(f[i:i + 4], "big")
        c = int.from_bytes(f[i + 4:i + 8], "big")
        assert raw == min(per * PKT, n - o)
        assert lz4_block_decode(f[i + 8:i + 8 + c], raw) == d[o:o + raw]
        i += 8 + c
        o += raw
        groups += 1
    assert o == n and groups == -(-n // (per * PKT))


def test_stream_ragged_writes_with_large_write():
    """Zero-length writes are no-ops; a write > MAX_INPUT flushes the buffered group, is sliced
    under one BE32 length header, and a trailing large write leaves close()'s BE32 0."""
    from oracle.oracle import hadoop_lz4_stream
    d = make_block("lowent", 4, 900_000).tobytes()
    writes = [1000, 0, 50_000, 600_000, 249_000]
    f = hadoop_lz4_stream(d, writes)
    assert hadoop_lz4_decode(f, len(d)) == d
    assert f[:4] == (51_000).to_bytes(4, "big")                 # first group: 1000 + 0 + 50,000
    f2 = hadoop_lz4_stream(d, [1000, 899_000])
    assert f2.endswith(b"\0\0\0\0") and hadoop_lz4_decode(f2, len(d)) == d


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_gpu_lz4_blocks_match_oracle(kind):
    """The GPU lz4_block (stream-mode Lz4Codec, one write) byte for byte against the oracle's r123
    restatement: table sizes byU16 (< 64 KiB + 11) and byU32, equal-hash batches (lowent, zeros,
    binary), catch-up across the segment start, multi-segment blocks."""
    from hdrf_amd.lib import Context
    from oracle.oracle import hadoop_lz4_stream
    ctx = Context(max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=16, arena_slots=16)
    for n in [13, 100, 4176, 65546, 65547, 70000, 261_100, 600_000]:
        for seed in (3, 4):
            d = make_block(kind, seed + n, n)
            assert ctx.stream_block_host(4, 1, d, [n]) == hadoop_lz4_stream(d, [n]), f"{kind} n={n} seed={seed}"
    ctx.close()
