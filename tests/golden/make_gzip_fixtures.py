"""Regenerate tests/golden/gzip_zlib.npz: gzip members written by this image's zlib 1.2.11
(level 6, windowBits 31, memLevel 8, default strategy = Hadoop GzipCodec's native
ZlibCompressor) for seeded blocks of every test kind.  Inputs are regenerated from
(kind, seed = 2000 + i, size) by tests/helpers.make_block; only the outputs are stored."""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from helpers import make_block  # noqa: E402

CASES = [("random", 33_000), ("zeros", 300_000), ("ff", 1), ("text", 40_000), ("lowent", 65_274),
         ("periodic", 200_003), ("sparse", 262_144), ("binary", 40_000), ("text", 0), ("text", 3)]


def main():
    assert zlib.ZLIB_RUNTIME_VERSION == "1.2.11", zlib.ZLIB_RUNTIME_VERSION
    out = {"kinds": np.array([k for k, _ in CASES]), "sizes": np.array([n for _, n in CASES], np.int64)}
    for i, (kind, n) in enumerate(CASES):
        d = make_block(kind, 2000 + i, n).tobytes()
        c = zlib.compressobj(6, zlib.DEFLATED, 31, 8, zlib.Z_DEFAULT_STRATEGY)
        out[f"out{i}"] = np.frombuffer(c.compress(d) + c.flush(), np.uint8)
    np.savez_compressed(os.path.join(HERE, "gzip_zlib.npz"), **out)


if __name__ == "__main__":
    main()
