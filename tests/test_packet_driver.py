"""The native packet-receive driver (tests/cpp/packet_driver.cpp): receiver threads calling the
C-ABI the JNI binding calls, one 64 KiB packet at a time (DN/BlockReceiver.java:877-896), each
packet mirrored downstream first (mirrorPacketTo, :635-641), blocks submitted in arrival order
(one per batch, or every block received in order since the last submit as one batch through
hdrf_submit_slots) and the durable containers
drained after every completed batch.  On the GPU every block's chunk END offsets, digests, is_new
and storeSize, and every container file the drains built, equal the sequential oracle's on the same
corpus; the mirror received every block intact."""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def _driver():
    import __graft_entry__ as ge
    return ge.build_packet_driver()


def test_packet_driver_compiles():
    assert os.access(_driver(), os.X_OK)


def _read_containers(path):
    disk = {}
    raw = open(path, "rb").read()
    o = 0
    while o < len(raw):
        cid, closed = np.frombuffer(raw, np.uint32, 2, o)
        n = int(np.frombuffer(raw, np.uint64, 1, o + 8)[0])
        disk[int(cid)] = (raw[o + 16:o + 16 + n], bool(closed))
        o += 16 + n
    return disk


@pytest.mark.gpu
@pytest.mark.parametrize("compressor,mirror,batch,mixed,nb,mib,cmax,slots", [
    (1, "socket", False, False, 6, 8, 1 << 20, 512),
    (2, "ring", True, True, 6, 8, 1 << 20, 512),
    # the bench's shape (config 5, the reference default compressor 2): 128 MiB blocks, 32 MiB
    # containers, 512 arena slots, mixed-entropy corpus, receive rounds handed over as batches
    (2, "ring", True, True, 8, 128, 1 << 25, 512),
])
def test_packet_driver_matches_oracle(tmp_path, compressor, mirror, batch, mixed, nb, mib, cmax, slots):
    from hdrf_amd.corpus import corpus_block_host, corpus_roots
    from oracle.oracle import Oracle
    exe = os.path.join(ROOT, "tools", "_build", "packet_driver")
    if not os.path.exists(exe):
        exe = _driver()
    args = [exe, str(nb), str(mib), "64", "4", "1", str(tmp_path), "--compressor", str(compressor), "--mirror", mirror,
            "--container-kib", str(cmax >> 10), "--index-log2", "20" if mib <= 8 else "24", "--arena-slots", str(slots)]
    args += ["--batch"] * batch + ["--mixed"] * mixed
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0
    line = json.loads(r.stdout.strip().splitlines()[-1])
    # warm-up + 1 timed step + the untimed step whose results OUT_DIR keeps
    assert line["mirror_ok"] is True and line["mirrored_bytes"] == 3 * nb * (mib << 20)
    # batched: the blocks received in order since the last submit go together (timing decides how many)
    assert (1 <= line["batches_per_step"] <= nb) if batch else line["batches_per_step"] == nb
    got = np.loadtxt(str(tmp_path / "blocks.txt"), dtype=np.int64).reshape(-1, 3)
    roots = corpus_roots(20251015, 500000, nb, mib)
    ora = Oracle(compressor=compressor, max_size=cmax)
    for b in range(nb):
        o = ora.reduce(corpus_block_host(20251015, roots, b, mib, 1 << 20, mixed=mixed), b)
        n = len(o["offsets"])
        assert got[b, 1] == n and got[b, 2] == o["store_size"], f"block {b}: {got[b]} vs oracle"
        raw = open(str(tmp_path / f"blk_{b}.bin"), "rb").read()
        assert len(raw) == n * (4 + 20 + 1)
        assert np.array_equal(np.frombuffer(raw, np.uint32, n, 0), o["offsets"]), f"block {b} offsets"
        assert np.array_equal(np.frombuffer(raw, np.uint8, n * 20, 4 * n).reshape(n, 20), o["digests"]), f"block {b} digests"
        assert np.array_equal(np.frombuffer(raw, np.uint8, n, 24 * n), o["is_new"]), f"block {b} is_new"
    # every container file the drains built (closed: raw or Lz4Codec; open: raw) is the oracle's
    disk = _read_containers(str(tmp_path / "containers.bin"))
    alloc = ora.allocator()
    n_cont = n_closed = 0
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, oc = ora.container(cid)
            if od is None:
                continue
            n_cont += 1
            n_closed += oc
            assert cid in disk, f"container {cid} never drained"
            assert disk[cid][0] == bytes(od) and disk[cid][1] == oc, f"container {cid} file differs"
    assert n_cont == len(disk) and n_closed >= 6, (n_cont, n_closed)
    print(f"{nb} x {mib} MiB blocks: {n_cont} container files ({n_closed} closed) equal the oracle's")
