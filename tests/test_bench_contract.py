"""bench.py bookkeeping that needs no GPU: the per-stream chains match the library's streams and
the committed PMC traffic is attached only to the workload it was measured on."""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

WANT = {"blocks": 512, "block_mib": 128, "batch": 32, "n_gpus": 1, "hasher": 0}


def _bench(monkeypatch, split=None):
    if split is None:
        monkeypatch.delenv("HDRF_SPLIT_B", raising=False)
    else:
        monkeypatch.setenv("HDRF_SPLIT_B", split)
    import bench
    return importlib.reload(bench)


def test_chains_follow_the_split_back_stage(monkeypatch):
    b = _bench(monkeypatch)
    assert list(b.CHAINS) == ["W: chunking", "A: SHA", "B: index", "B2: store", "L: LZ4"]
    assert "place(place_kernel)" in b.CHAINS["B2: store"]
    b = _bench(monkeypatch, "0")
    assert list(b.CHAINS) == ["W: chunking", "A: SHA", "B: index+store", "L: LZ4"]
    stages = [s for c in b.CHAINS.values() for s in c]
    assert len(stages) == len(set(stages))                # every stage timed on exactly one chain
    _bench(monkeypatch)


def test_traffic_is_matched_by_workload(monkeypatch):
    b = _bench(monkeypatch)
    d2, src2 = b.load_pmc(dict(WANT, workload="config2"))
    d4, src4 = b.load_pmc(dict(WANT, workload="config4"))
    assert src2 and src4 and src2 != src4
    assert d4["_config"]["workload"] == "config4"
    assert d2.get("_config", {}).get("workload", "config2") == "config2"
    assert "lz4_seg_kernel<false>" in d4 and "place_kernel<true>" in d2
    assert b.load_pmc(dict(WANT, workload="config5", blocks=128)) == ({}, None)


def test_named_kernels_have_committed_traffic(monkeypatch):
    """Every kernel the config-2 line names (its roofline entries) is in the newest config-2 traffic
    file, so a renamed kernel cannot silently drop the line's `traffic`."""
    b = _bench(monkeypatch)
    d, _ = b.load_pmc(dict(WANT, workload="config2"))
    for name, kern in b.KERNEL_OF.items():
        assert b.pmc_lookup(d, kern).get("hbm_bytes_per_launch"), (name, kern)


def test_fused_front_traffic_is_its_own(monkeypatch):
    """The fused front's PMC file is matched only when the line runs that front; the
    two-pass line keeps the two-pass file whatever sorts newest."""
    b = _bench(monkeypatch)
    d2, src2 = b.load_pmc(dict(WANT, workload="config2"))
    df, srcf = b.load_pmc(dict(WANT, workload="config2", front="fused"))
    assert src2 and srcf and src2 != srcf
    assert "lane_hash_kernel<5>" in df and "lane_hash_kernel<5>" not in d2
    assert "sha_carry_kernel<5>" in d2
