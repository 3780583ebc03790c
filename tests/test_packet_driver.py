"""The native packet-receive driver (tests/cpp/packet_driver.cpp): receiver threads calling the
C-ABI the JNI binding calls, one 64 KiB packet at a time (DN/BlockReceiver.java:877-896), blocks
submitted in arrival order and the durable containers drained after every completed block.  On the
GPU its per-block chunk counts and storeSize equal the sequential oracle's on the same corpus."""
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


@pytest.mark.gpu
def test_packet_driver_matches_oracle(tmp_path):
    from hdrf_amd.corpus import corpus_block_host, corpus_roots
    from oracle.oracle import Oracle
    exe = os.path.join(ROOT, "tools", "_build", "packet_driver")
    if not os.path.exists(exe):
        exe = _driver()
    nb, mib = 6, 8
    out = str(tmp_path / "blocks.txt")
    r = subprocess.run([exe, str(nb), str(mib), "64", "4", "1", out], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0
    got = np.loadtxt(out, dtype=np.int64).reshape(-1, 3)
    spb = mib
    roots = corpus_roots(20251015, 500000, nb, spb)
    ora = Oracle()
    for b in range(nb):
        o = ora.reduce(corpus_block_host(20251015, roots, b, spb, 1 << 20), b)
        assert got[b, 1] == len(o["offsets"]) and got[b, 2] == o["store_size"], f"block {b}: {got[b]} vs oracle"
