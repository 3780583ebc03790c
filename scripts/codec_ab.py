"""Stream-codec timings for A/B builds (HDRF_LIB_PATH selects the library): hdrf_stream_block
(encode, device-resident block) and hdrf_stream_file_decode (decode, file staged H2D) for codecs
0 (SnappyCodec), 3 (LzopCodec), 4 (Lz4Codec), 5 (GzipCodec) on one mixed block (text / binary /
random / low-entropy quarters); one warm call, then the best of three.  Prints MB/s of raw bytes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from helpers import make_block  # noqa: E402
from hdrf_amd.lib import Context  # noqa: E402


def best(f, reps=3):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        r = f()
        t.append(time.perf_counter() - t0)
    return min(t), r


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    n = mib << 20
    kinds = ["text", "binary", "random", "lowent"]
    a = np.concatenate([make_block(k, 7 + i, n // 4) for i, k in enumerate(kinds)])
    ctx = Context(max_block_bytes=n, max_batch_blocks=1, index_log2=20, arena_slots=16)
    dev = ctx.dev_alloc(n + 4096)
    ctx.h2d(dev, a)
    for codec, name in ((0, "snappy"), (3, "lzop"), (4, "lz4"), (5, "gzip")):
        ctx.stream_block(codec, 1, dev, n, n + 4096, [n])                  # warm
        te, f = best(lambda: ctx.stream_block(codec, 1, dev, n, n + 4096, [n]))
        ctx.stream_file_decode(codec, f, n)                                 # warm
        td, r = best(lambda: ctx.stream_file_decode(codec, f, n))
        assert r == a.tobytes(), name
        print(f"{name:7s} {mib} MiB  file {len(f) / n:.3f}x  encode {n / te / 1e6:9.1f} MB/s  decode {n / td / 1e6:9.1f} MB/s",
              flush=True)
    ctx.dev_free(dev)
    ctx.close()


if __name__ == "__main__":
    main()
