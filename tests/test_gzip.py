"""Stream-mode Gzip oracle (compressor == 5, DN/BlockReceiver.java:858-873,887-894,1238-1256):
Hadoop GzipCodec over the native ZlibCompressor (level 6, GZIP_FORMAT) writes one gzip member
per block, i.e. zlib's deflate of the whole block.  oracle/hdrf_gzip.c restates zlib 1.2.11's
deflate_slow + trees.c; it is pinned byte for byte against this image's zlib (1.2.11, the
library Hadoop's native codec links) and by round trips through zlib's inflate.  Committed
fixtures (tests/golden/gzip_zlib.npz, made by tests/golden/make_gzip_fixtures.py) keep the pin
when a different zlib is installed."""
import os
import zlib

import numpy as np
import pytest

from helpers import make_block
from oracle.oracle import gzip_stream

KINDS = ["random", "zeros", "ff", "text", "lowent", "periodic", "sparse", "binary"]
# window edges: 65274 = WSIZE + MAX_DIST (first slide), 65536 = window, 98304 = 3 half-windows
SIZES = [0, 1, 2, 3, 4, 100, 4096, 65_273, 65_274, 65_275, 65_536, 65_537, 98_304, 200_000]
ZLIB_1211 = zlib.ZLIB_RUNTIME_VERSION == "1.2.11"


def zlib_gzip(d):
    c = zlib.compressobj(6, zlib.DEFLATED, 31, 8, zlib.Z_DEFAULT_STRATEGY)
    return c.compress(d) + c.flush()


def test_golden_fixtures():
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "gzip_zlib.npz"))
    for i, (kind, n) in enumerate(zip(z["kinds"], z["sizes"])):
        d = make_block(str(kind), 2000 + i, int(n)).tobytes()
        assert gzip_stream(d) == z[f"out{i}"].tobytes(), f"fixture {i} ({kind}, {n})"


@pytest.mark.skipif(not ZLIB_1211, reason="pinned against zlib 1.2.11")
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", SIZES)
def test_matches_zlib(kind, n):
    d = make_block(kind, n * 7 + 1, n).tobytes()
    c = gzip_stream(d)
    assert c == zlib_gzip(d)
    assert zlib.decompress(c, 31) == d


@pytest.mark.skipif(not ZLIB_1211, reason="pinned against zlib 1.2.11")
def test_large_mixed_block_matches_zlib():
    """1 MiB of concatenated segments of every kind: dynamic, static and stored blocks, blocks
    longer than the window (stored ineligible), slides with pending lazy matches."""
    parts = [make_block(k, 31 + i, 131_072 + 977 * i) for i, k in enumerate(KINDS)]
    d = np.concatenate(parts).tobytes()
    assert gzip_stream(d) == zlib_gzip(d)


def test_gzip_member_framing():
    d = make_block("text", 9, 70_000).tobytes()
    c = gzip_stream(d)
    assert c[:10] == bytes([0x1F, 0x8B, 8, 0, 0, 0, 0, 0, 0, 3])    # zlib's gzip header (OS_CODE 3)
    assert int.from_bytes(c[-8:-4], "little") == zlib.crc32(d)
    assert int.from_bytes(c[-4:], "little") == len(d)
