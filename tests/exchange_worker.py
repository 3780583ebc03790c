"""Exchange worker for tests/test_node.py: world-size-2 gloo on CPU tensors
(test_exchange_gloo_cpu_world2), or the RCCL branch on GPU tensors (HDRF_XW_BACKEND=nccl,
test_exchange_rccl_gpu: list all_to_all, all_gather, send/recv and broadcast over RCCL)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hdrf_amd.lib import ALLOC_STATE_BYTES  # noqa: E402
from hdrf_amd.node import Exchange  # noqa: E402


def main():
    nccl = os.environ.get("HDRF_XW_BACKEND") == "nccl"
    dev = None
    if nccl:
        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    r, G = dist.get_rank(), dist.get_world_size()
    xc = Exchange(G, r, dev)
    assert xc.nccl == nccl
    cap, w = 50, 3
    send = torch.full((G * cap * w,), -1, dtype=torch.int32)
    counts = np.array([(r * 7 + d * 3) % 11 + d for d in range(G)], np.int64)
    for d in range(G):
        for i in range(int(counts[d])):
            send[(d * cap + i) * w:(d * cap + i + 1) * w] = torch.tensor([r, d, i], dtype=torch.int32)
    rc = xc.counts(counts)
    expect_rc = np.array([(s * 7 + r * 3) % 11 + r for s in range(G)], np.int64)
    assert np.array_equal(rc, expect_rc), (rc, expect_rc)
    recv = torch.full((G * cap * w,), -1, dtype=torch.int32)
    if nccl:
        send, recv = send.to(dev), recv.to(dev)
    xc.records(send, recv, counts, rc, cap, w)
    recv = recv.cpu()
    for s in range(G):
        for i in range(int(rc[s])):
            got = recv[(s * cap + i) * w:(s * cap + i + 1) * w].tolist()
            assert got == [s, r, i], (s, i, got)
        assert int(recv[(s * cap + int(rc[s])) * w]) == -1      # nothing past the count
    # allocator hand-off: each rank adds its rank+1 to byte 0; everyone sees the last rank's state
    start = np.zeros(ALLOC_STATE_BYTES, np.uint8)

    def flush(a_in):
        a = np.array(a_in if a_in is not None else start, np.uint8)
        a[0] += r + 1
        a[1 + r] = 0xA0 + r
        return a
    fin = xc.chain_alloc(start, flush)
    assert int(fin[0]) == G * (G + 1) // 2 and all(int(fin[1 + q]) == 0xA0 + q for q in range(G)), fin[:4]
    # descriptors of different lengths for the allocator scan
    got = xc.all_gather_i64(np.arange(3 + 5 * r, dtype=np.int64) * (r + 1))
    assert [g.tolist() for g in got] == [(np.arange(3 + 5 * q) * (q + 1)).tolist() for q in range(G)], got
    # equal-size device buffers (the packed flush descriptors of the device allocator scan)
    fs = torch.arange(40, dtype=torch.uint8) + 50 * r
    fr = torch.zeros(G * 40, dtype=torch.uint8)
    if nccl:
        fs, fr = fs.to(dev), fr.to(dev)
    xc.all_gather_dev(fs, fr)
    assert fr.cpu().tolist() == [int(x) for q in range(G) for x in (torch.arange(40) + 50 * q).tolist()]
    print("exchange ok", r, "nccl" if nccl else "gloo", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
