"""Shared test data generators and comparisons (test infrastructure)."""
import numpy as np

from hdrf_amd.corpus import mix64


def prng_bytes(seed, n):
    """Deterministic bytes from splitmix64 (stable across numpy versions)."""
    nw = (n + 7) // 8
    with np.errstate(over="ignore"):
        w = mix64(np.uint64(seed) * np.uint64(0x9E3779B97F4A7C15) + np.arange(nw, dtype=np.uint64))
    return w.view(np.uint8)[:n].copy()


def make_block(kind, seed, n):
    r = prng_bytes(seed, n)
    if kind == "random":
        return r
    if kind == "zeros":
        return np.zeros(n, np.uint8)
    if kind == "ff":
        return np.full(n, 0xFF, np.uint8)
    if kind == "text":           # ASCII-ish alphabet: window max is rarely 127
        alpha = np.frombuffer(b"etaoinshrdlucmfwypvbgkjqxz ETAOIN.,\n0123456789", np.uint8)
        return alpha[r % len(alpha)]
    if kind == "lowent":         # 4-symbol alphabet
        return (r & 3).astype(np.uint8) + 60
    if kind == "periodic":       # exact period -> speculative chains never meet (fallback)
        pat = prng_bytes(seed + 1, 1000)
        return np.resize(pat, n)
    if kind == "sparse":         # zero runs with random islands
        out = np.zeros(n, np.uint8)
        for i in range(0, n, 65536):
            out[i:i + 4096] = r[i:i + 4096]
        return out
    if kind == "binary":         # small-magnitude little-endian int32 records
        v = (r.view(np.uint8)[: n - n % 4].view(np.int32) % 200).astype(np.int32)
        b = v.view(np.uint8)
        return np.concatenate([b, r[: n - b.size]])
    raise ValueError(kind)


def compare_block(g, o, tag=""):
    assert len(g["offsets"]) == len(o["offsets"]), f"{tag}: chunk count {len(g['offsets'])} vs {len(o['offsets'])}"
    bad = np.nonzero(g["offsets"] != o["offsets"])[0]
    assert bad.size == 0, f"{tag}: first boundary mismatch at chunk {bad[:5]}: {g['offsets'][bad[:5]]} vs {o['offsets'][bad[:5]]}"
    assert np.array_equal(g["digests"], o["digests"]), f"{tag}: digests differ"
    assert np.array_equal(g["is_new"], o["is_new"]), f"{tag}: is_new differs"
    assert g["store_size"] == o["store_size"], f"{tag}: storeSize {g['store_size']} vs {o['store_size']}"
    # container placement of new chunks == the location each chunk SETs (chunkMeta.getMeta)
    if "values" in o and "container_id" in g and o["store_size"] > 0:
        v = o["values"].astype(np.uint32)
        cid = (v[:, 1] << 16) | (v[:, 2] << 8) | v[:, 3]
        start = ((v[:, 10] & 0xF0) << 20) | (v[:, 4] << 16) | (v[:, 5] << 8) | v[:, 6]
        m = o["is_new"].astype(bool)
        assert np.array_equal(g["container_id"][m], cid[m]), f"{tag}: container ids differ"
        assert np.array_equal(g["container_pos"][m], start[m]), f"{tag}: container positions differ"


def compare_state(ctx, ora, block_ids, tag="", containers=True):
    gk, gv = ctx.index_dump()
    ok, ov = ora.index_dump()
    assert gk.shape == ok.shape, f"{tag}: index size {gk.shape[0]} vs {ok.shape[0]}"
    assert np.array_equal(gk, ok), f"{tag}: index keys differ"
    bad = np.nonzero((gv != ov).any(axis=1))[0]
    assert bad.size == 0, f"{tag}: index values differ at {bad[:5]}: {gv[bad[:3]]} vs {ov[bad[:3]]}"
    assert ctx.allocator() == ora.allocator(), f"{tag}: allocator {ctx.allocator()} vs {ora.allocator()}"
    for bid in block_ids:
        assert ctx.recipe(bid) == ora.recipe(bid), f"{tag}: recipe {bid} differs"
        assert ctx.block_length(bid) == int.from_bytes(ora.recipe(bid)[:4], "big")
    # every container the oracle wrote
    alloc = ora.allocator()
    if alloc and containers:
        ids = [int.from_bytes(alloc[3 * t:3 * t + 3], "big") for t in range(3)]
        for t in range(3):
            base = t << 22
            for cid in range(base, ids[t] + 1):
                od, oc = ora.container(cid)
                gd, gc = ctx.container(cid)
                if od is None:
                    continue
                assert gd is not None, f"{tag}: container {cid} missing"
                assert gd == od, f"{tag}: container {cid} bytes differ ({len(gd)} vs {len(od)})"
                assert gc == oc, f"{tag}: container {cid} closed flag"
