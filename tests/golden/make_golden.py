"""Generate the golden fixtures under tests/golden/ from the CPU oracle.

Run: python tests/golden/make_golden.py
Each case is a sequence of blocks (regenerated from (kind, seed, size) specs with
tests/helpers.make_block) reduced in order by one DataNode.  Every oracle output is first
cross-checked against the independent pure-Python transliteration (oracle/pyref.py) and
SHA digests against hashlib; then offsets / is_new / store sizes are stored verbatim and
digests, 11-byte values, the final index, recipes and containers as SHA-256 checksums.
The Java reference cannot run here (no JDK/Redis), so these fixtures pin the restatement,
not the running reference.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import make_block  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import pyref as P  # noqa: E402

CASES = {
    "mixed_sha1": dict(hasher=0, max_size=1 << 25, blocks=[
        ("random", 1, 200_000), ("random", 1, 200_000), ("text", 2, 150_000), ("zeros", 3, 50_000),
        ("ff", 4, 30_000), ("random", 5, 0), ("random", 6, 701), ("random", 7, 702), ("random", 8, 1500),
        ("lowent", 9, 120_000), ("periodic", 10, 90_000), ("sparse", 11, 300_000), ("binary", 12, 100_000)]),
    "mixed_sha224": dict(hasher=1, max_size=1 << 25, blocks=[
        ("random", 21, 180_000), ("text", 22, 100_000), ("random", 21, 180_000), ("zeros", 23, 20_000),
        ("binary", 24, 64_000)]),
    "flush_small_containers": dict(hasher=0, max_size=1_000_002 + 48_574, blocks=[
        ("random", 31, 1_100_000), ("random", 32, 900_000), ("random", 31, 1_100_000), ("text", 33, 700_000),
        ("random", 34, 1_500_000)]),
}


def sha(b):
    return hashlib.sha256(bytes(b)).hexdigest()


def build_case(name, spec):
    ora = O.Oracle(hasher=spec["hasher"], compressor=1, max_size=spec["max_size"])
    ref = P.PyRef(hasher=spec["hasher"], max_size=spec["max_size"])
    out = {"hasher": spec["hasher"], "max_size": spec["max_size"], "blocks": []}
    arrays = {}
    for i, (kind, seed, size) in enumerate(spec["blocks"]):
        data = make_block(kind, seed, size)
        bid = 100 + i
        o = ora.reduce(data, bid)
        p = ref.reduce(bytes(data), bid)
        assert list(o["offsets"]) == p["offsets"], (name, i)
        assert [bytes(d) for d in o["digests"]] == p["digests"], (name, i)
        assert list(o["is_new"]) == p["is_new"] and o["store_size"] == p["store_size"], (name, i)
        hf = hashlib.sha1 if spec["hasher"] == 0 else hashlib.sha224
        prev = 0
        for end, d in zip(o["offsets"], o["digests"]):
            assert hf(bytes(data[prev:end])).digest() == bytes(d)
            prev = int(end)
        arrays[f"b{i}_offsets"] = o["offsets"]
        arrays[f"b{i}_is_new"] = o["is_new"]
        out["blocks"].append({"kind": kind, "seed": seed, "size": size, "block_id": bid,
                              "n": int(len(o["offsets"])), "store_size": int(o["store_size"]),
                              "digests_sha256": sha(o["digests"]), "values_sha256": sha(o["values"]),
                              "input_sha256": sha(data)})
    keys, vals = ora.index_dump()
    assert len(keys) == sum(1 for k in ref.redis if len(k) == ora.H)
    for k, v in zip(keys, vals):
        assert ref.redis[bytes(k)] == bytes(v)
    out["index_count"] = int(len(keys))
    out["index_sha256"] = sha(np.concatenate([keys.reshape(-1), vals.reshape(-1)]))
    out["allocator"] = ora.allocator().hex()
    assert ora.allocator() == ref.redis[b"blockID"]
    out["recipes_sha256"] = {str(b["block_id"]): sha(ora.recipe(b["block_id"])) for b in out["blocks"]}
    conts = {}
    alloc = ora.allocator()
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            d, closed = ora.container(cid)
            if d is not None:
                assert d == bytes(ref.files[cid]) and closed == (cid in ref.closed)
                conts[str(cid)] = {"len": len(d), "closed": closed, "sha256": sha(d)}
    out["containers"] = conts
    return out, arrays


def main():
    for name, spec in CASES.items():
        meta, arrays = build_case(name, spec)
        with open(os.path.join(HERE, f"{name}.json"), "w") as f:
            json.dump(meta, f, indent=1, sort_keys=True)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrays)
        print(name, len(meta["blocks"]), "blocks,", meta["index_count"], "index entries,",
              len(meta["containers"]), "containers")


if __name__ == "__main__":
    main()
