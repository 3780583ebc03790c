"""Per-phase LZ4 parse time (profiling build, -DHDRF_LZ4_PROF, hdrf_amd/_build_prof): shader-clock
cycles summed over waves for each phase of lz4_block, per config-4 kind, at ~1 wave per CU (64 MiB
block, 257 pieces) and at full occupancy (2 GiB, 8225 pieces); scripts/r02_lzp.sh."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("HDRF_LIB_PATH", os.path.join(ROOT, "hdrf_amd", "_build_prof", "libhdrf.so"))
sys.path.insert(0, ROOT)
from hdrf_amd.corpus import segment_kind  # noqa: E402
from hdrf_amd.lib import Context, load  # noqa: E402

PH = ["search batch", "catch-up+literals", "chain top+extension", "tokens+table", "Cw load+compare",
      "(unused)", "last literals", "(unused)"]


def main():
    L = load()
    L.hdrf_debug_lz4_prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 16)()
    seg = 1 << 20
    sizes = [int(x) for x in os.environ.get("LZP_MIB", "64,2048").split(",")]
    mx = max(sizes)
    ctx = Context(max_block_bytes=64 << 20, max_batch_blocks=1, index_log2=20, arena_slots=16)
    dev = ctx.dev_alloc((mx << 20) + 4096)
    for kind in (1, 2):
        roots = np.array([r for r in range(1, 40 * mx) if segment_kind(r) == kind][:mx], np.uint32)
        ctx.corpus_fill(dev, roots, 1, mx, seg, 7, mixed=True)
        ctx.synchronize()
        for mib in sizes:
            n = mib << 20
            L.hdrf_debug_lz4_prof(buf, 1)
            ctx.stream_block(4, 1, dev, n, n + 4096, [n])
            L.hdrf_debug_lz4_prof(buf, 1)
            v = list(buf)
            tot = sum(v[:8])
            nb, nf, nc = v[8], v[9], v[10]
            print(f"kind {kind} {mib} MiB: total {tot / 1e9:.3f} Gcyc; search batches {nb}, found {nf}, chained {nc}; "
                  f"cyc/seq {tot / max(1, nf + nc):.0f}", flush=True)
            for i, name in enumerate(PH):
                if v[i]:
                    per = v[i] / max(1, (nb if i == 0 else nf if i == 1 else nf + nc if i in (2, 3) else nf + nc))
                    print(f"   {name:22s} {v[i] / tot:6.3f}  {per:8.0f} cyc/event", flush=True)
    ctx.dev_free(dev)
    ctx.close()


if __name__ == "__main__":
    main()
