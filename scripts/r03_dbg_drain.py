"""Debug: in-flight drain scenario variants (which ingredient breaks block chunking)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
from test_boundary import _blocks
from hdrf_amd.lib import Context
from oracle.oracle import Oracle, chunk

def run(drain, retain, pinned, depth=3, comp=1):
    cmax = 1 << 20
    blocks = _blocks(71 + comp, 20, 2 << 20, dup_div=8)
    ids = [6500 + i for i in range(len(blocks))]
    ctx = Context(compressor=comp, container_max=cmax, max_block_bytes=4 << 20, max_batch_blocks=1,
                  index_log2=20, arena_slots=64, retain_containers=retain)
    if pinned:
        hb = ctx.host_alloc(len(blocks) * (2 << 20))
        for k, b in enumerate(blocks):
            hb[k * (2 << 20):(k + 1) * (2 << 20)] = b
        ptrs = [hb.ctypes.data + k * (2 << 20) for k in range(len(blocks))]
    else:
        ptrs = [b.ctypes.data for b in blocks]
    bad = []
    pend = []
    def check():
        ctx.wait_batch()
        k = pend.pop(0)
        g = ctx.batch_result(0)["offsets"]
        o = chunk(blocks[k])
        if len(g) != len(o) or not np.array_equal(g, o):
            n = min(len(g), len(o))
            d = np.nonzero(g[:n] != o[:n])[0]
            bad.append((k, len(g), len(o), int(d[0]) if d.size else n, int(o[d[0]]) if d.size else -1))
        if drain:
            ctx.drain_containers(buf_bytes=1 << 20)
    for k in range(len(blocks)):
        ctx.submit_host([ptrs[k]], [2 << 20], [ids[k]])
        pend.append(k)
        if len(pend) == depth:
            check()
    while pend:
        check()
    ctx.close()
    print("drain=%d retain=%d pinned=%d depth=%d comp=%d -> bad %s" % (drain, retain, pinned, depth, comp, bad[:4]), flush=True)

for args in [(1, 1, 0), (0, 1, 0), (0, 0, 0), (1, 1, 1), (0, 0, 1)]:
    run(*args)
run(0, 0, 0, depth=1)
