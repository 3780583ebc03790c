"""GzipCodec read side throughput: hdrf_stream_file_decode(5) on block files of the stream-mode
compressor 5 (one gzip member per block, DN/BlockReceiver.java:858-873) vs this host's zlib.
Wall clock per call (file H2D + inflate + CRC), and the kernel alone under rocprofv3."""
import sys
import time
import zlib

import numpy as np

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from hdrf_amd.lib import Context  # noqa: E402
from tests.helpers import make_block  # noqa: E402


def main():
    sizes = [int(a) for a in sys.argv[1:]] or [1 << 20, 16 << 20, 64 << 20]
    ctx = Context(max_block_bytes=128 << 20, max_batch_blocks=1, index_log2=20, arena_slots=16)
    for kind in ("text", "binary", "random"):
        for n in sizes:
            a = make_block(kind, 5, n).tobytes()
            c = zlib.compressobj(6, zlib.DEFLATED, 31)
            f = np.frombuffer(c.compress(a) + c.flush(), np.uint8)
            out = ctx.stream_file_decode(5, f, n)
            assert out == a
            t = time.perf_counter()
            reps = 3
            for _ in range(reps):
                ctx.stream_file_decode(5, f, n)
            g = (time.perf_counter() - t) / reps
            t = time.perf_counter()
            zlib.decompress(f.tobytes(), 31)
            z = time.perf_counter() - t
            print(f"{kind:7s} {n >> 20:4d} MiB file {f.size / n:.3f}x  gpu {n / g / 1e6:8.1f} MB/s  "
                  f"zlib(1 core) {n / z / 1e6:8.1f} MB/s", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
