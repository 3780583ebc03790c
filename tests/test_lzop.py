"""Stream-mode compressor 3 (hadoop-lzo LzopCodec; DN/BlockReceiver.java:836-845 write,
DN/DataConstructor.java:140-166 read).

The oracle (oracle/hdrf_lzo.c) restates LZO 2.10 lzo1x_1_compress (x86-64 build) and hadoop-lzo's
LzopOutputStream framing.  Neither hadoop-lzo nor liblzo2 is in this image, so the compressed bytes
are parity UNPINNED against the reference; the restatement is checked here by its own LZO1X decoder
(round trips over the edge sizes of the 49,152-B sub-blocks and the 245,693-B stream blocks), the
LZO1X format rules, and the lzop header against zlib's Adler-32; the GPU path (lzo.hip) is compared
with it byte for byte and decodes the oracle's files.
"""
import struct
import zlib

import numpy as np
import pytest

from helpers import make_block
from oracle.oracle import lzo1x_1, lzo1x_decode, lzop_decode, lzop_stream

KINDS = ["random", "zeros", "text", "lowent", "periodic", "sparse", "binary", "ff"]
SIZES = [0, 1, 3, 4, 17, 20, 21, 25, 31, 32, 33, 100, 1000, 49151, 49152, 49153, 98304, 98305, 245692, 245693]
MAX_IN = 262144 - (262144 // 16 + 64 + 3)          # LzopOutputStream MAX_INPUT_SIZE


def lzop_blocks(f):
    """(raw length, stored length) of every block of an lzop file written with flags 0."""
    assert f[:9] == b"\x89LZO\x00\r\n\x1a\n"
    pos, out = 9 + 25 + f[9 + 24] + 4, []
    while True:
        ul, = struct.unpack(">I", f[pos:pos + 4])
        pos += 4
        if ul == 0:
            break
        cl, = struct.unpack(">I", f[pos:pos + 4])
        out.append((ul, cl))
        pos += 4 + cl
    assert pos == len(f)
    return out


@pytest.mark.parametrize("kind", KINDS)
def test_lzo1x_1_round_trip(kind):
    for n in SIZES:
        d = make_block(kind, 7 + n, n)
        c = lzo1x_1(d)
        assert np.array_equal(lzo1x_decode(c, n), d), f"{kind} n={n}"
        assert bytes(c[-3:]) == b"\x11\x00\x00"                     # M4 end-of-stream marker
        assert len(c) <= n + n // 16 + 64 + 3                       # lzo1x worst case


def test_lzo1x_1_small_inputs_are_literal_only():
    """<= 20 bytes, and 21..31 bytes (lzo's overflow guard: t + ll < 32), are one literal run in the
    first-byte form 17 + n; a zero-length input is the end marker alone."""
    assert bytes(lzo1x_1(np.zeros(0, np.uint8))) == b"\x11\x00\x00"
    for n in (1, 5, 20, 21, 31):
        d = make_block("zeros", 1, n)
        assert bytes(lzo1x_1(d)) == bytes([17 + n]) + bytes(d) + b"\x11\x00\x00", n
    assert len(lzo1x_1(np.zeros(32, np.uint8))) < 32 + 4                # 32 bytes: the parse runs


def test_lzop_header_fields_and_adler32():
    f = lzop_stream(np.zeros(0, np.uint8), [], mtime=0x5f5e1000)
    body = (b"\x10\x10" + b"\x20\xa0" + b"\x09\x40" + bytes([1, 5]) + struct.pack(">I", 0) + struct.pack(">I", 0x81a4)
            + struct.pack(">I", 0x5f5e1000) + struct.pack(">I", 0) + b"\x00")
    assert bytes(f) == b"\x89LZO\x00\r\n\x1a\n" + body + struct.pack(">I", zlib.adler32(body)) + b"\x00\x00\x00\x00"


def test_lzop_stream_block_structure():
    """Blocks are cut like BlockCompressorStream: 64,512-B packets give 3 per block; a write larger
    than MAX_INPUT is cut into MAX_INPUT slices, each its own [raw][stored] block; incompressible
    blocks are stored raw (stored == raw); close() ends with BE32 0."""
    d = make_block("binary", 9, 2_000_000)
    f = bytes(lzop_stream(d, [64512] * 12 + [len(d) - 64512 * 12]))
    bl = lzop_blocks(f)
    assert [u for u, _ in bl[:4]] == [3 * 64512] * 4
    assert bl[4][0] == MAX_IN and sum(u for u, _ in bl) == len(d)
    assert all(c < u for u, c in bl)
    assert np.array_equal(lzop_decode(f, len(d)), d)
    r = make_block("random", 9, 600_000)
    fr = bytes(lzop_stream(r, [len(r)]))
    assert lzop_blocks(fr) == [(MAX_IN, MAX_IN), (MAX_IN, MAX_IN), (600_000 - 2 * MAX_IN, 600_000 - 2 * MAX_IN)]
    assert np.array_equal(lzop_decode(fr, len(r)), r)


def test_lzop_decode_rejects_corruption():
    d = make_block("text", 2, 300_000)
    f = bytearray(lzop_stream(d, [len(d)]))
    bad = bytearray(f)
    bad[20] ^= 1                                                    # header byte: checksum mismatch
    with pytest.raises(ValueError):
        lzop_decode(np.frombuffer(bytes(bad), np.uint8), len(d))
    with pytest.raises(ValueError):
        lzop_decode(np.frombuffer(bytes(f[:-7]), np.uint8), len(d))  # truncated


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_gpu_lzop_matches_oracle(kind):
    """hdrf_stream_block(3) byte for byte against the oracle: sub-block edges, the 21..31-byte guard,
    multi-block files, raw (incompressible) blocks; then the GPU decodes every file back."""
    from hdrf_amd.lib import Context
    ctx = Context(max_block_bytes=4 << 20, max_batch_blocks=1, index_log2=16, arena_slots=16)
    ctx.set_lzop_mtime(1234567)
    for n in SIZES + [600_000]:
        d = make_block(kind, 11 + n, n)
        g = ctx.stream_block_host(3, 1, d, [n] if n else [])
        o = bytes(lzop_stream(d, [n] if n else [], mtime=1234567))
        assert g == o, f"{kind} n={n}"
        assert bytes(ctx.stream_file_decode(3, g, n)) == d.tobytes(), f"{kind} n={n} decode"
    ctx.close()


@pytest.mark.gpu
def test_gpu_lzop_packet_writes_and_corruption():
    """Packet-sized writes (64,512 B), ragged writes with one larger than MAX_INPUT, an empty block;
    a corrupted LZO1X end marker is an error (LzopCodec files written with flags 0 carry no block
    checksums, so only structural corruption is detectable)."""
    from hdrf_amd.lib import Context, HdrfError
    ctx = Context(max_block_bytes=8 << 20, max_batch_blocks=1, index_log2=16, arena_slots=16)
    d = np.concatenate([make_block(k, 5, 700_000) for k in ("text", "random", "lowent", "binary")])
    for w in ([64512] * (len(d) // 64512) + [len(d) % 64512], [1, 700, 300_000, 1_000_000, len(d) - 1_300_701]):
        g = ctx.stream_block_host(3, 2, d, w)
        assert g == bytes(lzop_stream(d, w)), w[:3]
        assert bytes(ctx.stream_file_decode(3, g, len(d))) == d.tobytes()
    assert ctx.stream_block_host(3, 3, np.zeros(0, np.uint8), []) == bytes(lzop_stream(np.zeros(0, np.uint8), []))
    g = bytearray(ctx.stream_block_host(3, 4, d, [len(d)]))
    bl = lzop_blocks(bytes(g))
    first_compressed = next(i for i, (u, c) in enumerate(bl) if c < u)
    pos = 9 + 25 + 4 + sum(8 + c for _, c in bl[:first_compressed]) + 8
    g[pos + bl[first_compressed][1] - 1] = 1                       # the block's end marker 11 00 00 -> 11 00 01
    with pytest.raises(HdrfError):
        ctx.stream_file_decode(3, bytes(g), len(d))
    ctx.close()


def test_lzop_fixed_bytes_fixture():
    """The committed file bytes (tests/golden/lzop_fixed.npz, made by make_lzop_fixture.py): the
    oracle must still write exactly them, and they decode to the input."""
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "lzop_fixed.npz"))
    data, f, mtime = z["data"], z["lzop"], int(z["mtime"][0])
    assert np.array_equal(lzop_stream(data, [len(data)], mtime=mtime), f)
    assert np.array_equal(lzop_decode(f, len(data)), data)
    assert f[:9].tobytes() == b"\x89LZO\x00\r\n\x1a\n"
    assert mtime.to_bytes(4, "big") in f[9:40].tobytes()                 # header mtime field


@pytest.mark.gpu
def test_lzop_fixed_bytes_fixture_gpu():
    """The GPU LzopCodec writes the committed fixture's bytes (same mtime) and reads them back."""
    import os
    from hdrf_amd.lib import Context
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "lzop_fixed.npz"))
    data, f, mtime = z["data"], z["lzop"], int(z["mtime"][0])
    ctx = Context(max_block_bytes=1 << 20, max_batch_blocks=1, index_log2=16, arena_slots=8)
    ctx.set_lzop_mtime(mtime)
    g = ctx.stream_block_host(3, 1, data, [len(data)])
    assert np.array_equal(np.frombuffer(bytes(g), np.uint8), f)
    assert np.array_equal(np.frombuffer(bytes(ctx.stream_file_decode(3, g, len(data))), np.uint8), data)
    ctx.close()
