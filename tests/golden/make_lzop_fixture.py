"""Fixed-bytes LzopCodec fixture: the lzop header and one small compressed block, as the
oracle's restatement of hadoop-lzo LzopOutputStream + LZO 2.10 lzo1x_1 writes them today.  Parity
vs hadoop-lzo stays UNPINNED (no hadoop-lzo or liblzo2 here); the fixture only freezes the bytes so
a later change to the oracle cannot move the GPU output along with it unnoticed.

Run from the repo root: python tests/golden/make_lzop_fixture.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import make_block  # noqa: E402
from oracle.oracle import lzop_stream  # noqa: E402


def main():
    data = np.concatenate([make_block("text", 3, 3000), make_block("random", 4, 500), np.zeros(700, np.uint8)])
    f = lzop_stream(data, [len(data)], mtime=1700000000)
    np.savez(os.path.join(ROOT, "tests", "golden", "lzop_fixed.npz"), data=data, lzop=f,
             mtime=np.array([1700000000], np.uint32))
    print(len(data), "->", len(f), "bytes")


if __name__ == "__main__":
    main()
