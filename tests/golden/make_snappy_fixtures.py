"""Generate tests/golden/snappy_pyarrow.npz: seeded inputs (tests/helpers.make_block) and their snappy raw encodings made by
the snappy library bundled in pyarrow (snappy::RawCompress, level 1) -- the published compressor
the oracle's restatement (oracle/hdrf_oracle.c, sn_fragment) is pinned against.  Hadoop's
SnappyCodec calls the same function through its native SnappyCompressor.

    python tests/golden/make_snappy_fixtures.py
"""
import os
import sys

import numpy as np
import pyarrow as pa

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from helpers import make_block  # noqa: E402

CASES = [("random", 0), ("random", 14), ("random", 15), ("text", 16), ("text", 255), ("text", 256),
         ("lowent", 257), ("zeros", 65_535), ("lowent", 65_536), ("text", 65_537), ("binary", 100_000),
         ("periodic", 131_072), ("sparse", 150_000), ("ff", 70_000), ("lowent", 218_422), ("text", 218_422)]


def main():
    arrs = {}
    for i, (kind, n) in enumerate(CASES):
        d = make_block(kind, 1000 + i, n).tobytes()
        arrs[f"out{i}"] = np.frombuffer(pa.compress(d, codec="snappy", asbytes=True), np.uint8)
    arrs["kinds"] = np.array([k for k, _ in CASES])      # inputs: make_block(kind, 1000 + i, n)
    arrs["sizes"] = np.array([n for _, n in CASES], np.int64)
    np.savez_compressed(os.path.join(os.path.dirname(__file__), "snappy_pyarrow.npz"), **arrs)
    print("snappy", pa.__version__, len(CASES), "cases")


if __name__ == "__main__":
    main()
