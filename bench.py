#!/usr/bin/env python3
"""bench.py — HDRF per-block reduction throughput on MI355X (BASELINE config 2).

Workload (per GPU): a synthetic corpus of 512 blocks x 128 MiB (64 GiB) resident in HBM,
1 MiB segments, 50% of them copies of a segment of an EARLIER block (cross-block
duplicates).  One step = one DataNode reducing the whole corpus in block
order from a fresh index: window-max chunking -> SHA-1 -> GPU index (exact HDRF dedup
semantics) -> container placement + gather into the container arena, in batches of 32
blocks (4 GiB), four batches in flight, steps back to back (hdrf_reset_async).  value = logical bytes reduced per second over all ranks (GB = 1e9 B).

Multi-GPU (`torch.distributed.run`, BASELINE config 3): the GPUs of the node are ranks of ONE
reduction, as the DataNodes of one host share one Redis, allocator and chunkDir in the reference
(DN/DataDeduplicator.java:119,165-172): a global corpus of N x 512 blocks sharded by block, each
global batch takes --batch (32) blocks from every rank, and the fingerprint index is partitioned by digest
prefix with three RCCL all-to-alls per batch over xGMI (hdrf_amd/node.py).  Work per GPU is
fixed as N grows: scaling is weak.  (HDRF_BENCH_SAME_DEVICE=1 puts every rank on cuda:0 over gloo:
a one-GPU rehearsal of the multi-rank path, not a measurement.)

The line also carries the dominant kernel's roofline (HIP events on the library's stream)
and the CPU oracle timed on this host on a bounded sample of the same corpus, whose
per-block storeSize must equal the GPU's (bit-exact dedup ratio check).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "logical GB/s reduced per node (1/2/4/8 GPUs) at 50% dup, bit-exact dedup ratio"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_WI_NS = 1033.0       # v_add_u32 wave-instructions/ns, chip-wide (tools/valu_peak.hip)
KERNEL_OF = {"gmax(gmax_kernel)": "gmax_kernel" if os.environ.get("HDRF_GMAX_V", "2") == "1" else "gmax2_kernel",
             "walk(lane_walk_kernel)": "lane_walk_kernel",
             "sha(sha_chunk_kernel)": "sha_carry_kernel" if os.environ.get("HDRF_SHA_CARRY", "1") not in ("", "0")
             else "sha_chunk_kernel", "place(place_kernel)": "place_kernel"}
# the fused chunk + fingerprint front (HDRF_FUSED, hdrf_amd/csrc/lanehash.hip; mirrors api.hip fused_front()):
# the walk slot times lane_hash_kernel, the granule slot is empty, the SHA slot is the listed fix-up
FUSED = os.environ.get("HDRF_FUSED", "0") not in ("", "0")
if FUSED:
    KERNEL_OF["walk(lane_walk_kernel)"] = "lane_hash_kernel"
# stages per stream (hdrf_amd/csrc/api.hip submit): W chunking, A fingerprints, B index (claim ..
# finalize), B2 store (scans, flush, place; on stream B itself with HDRF_SPLIT_B=0), L the LZ4 pass
# of closed containers (compressor 2; two LZ4 streams alternating by batch)
_INDEX = ["index_claim(idx_claim_kernel)", "index_apply(idx_apply_kernel)", "index_slow_decide(idx_slow/decide)"]
_STORE = ["scan(tile/chunk_scan)", "flush(flush_kernel)", "place(place_kernel)"]
CHAINS = {"W: chunking": ["gmax(gmax_kernel)", "walk(lane_walk_kernel)", "stitch(repair/path/count/scan/copy/fallback)"],
          "A: SHA": ["sha(sha_chunk_kernel)", "sha_tail(none: padding inside the sha kernel)"]}
if os.environ.get("HDRF_SPLIT_B", "1") not in ("", "0"):
    CHAINS.update({"B: index": _INDEX, "B2: store": _STORE})
else:
    CHAINS["B: index+store"] = _INDEX + _STORE
CHAINS["L: LZ4"] = ["compress(lz4_seg/lz4_pack)"]
# node-global ranks (N > 1, hdrf_amd/node.py): the front on W / A / X, the back phases and the gaps the
# exchanges fill on stream B, the arena copy on B2 (api.hip gx_collect)
CHAINS_GX = {"W: chunking": CHAINS["W: chunking"], "A: SHA": ["sha(sha_chunk_kernel)"],
             "X: local aggregation": ["gx_local(scratch claim/apply/decide + gx_emit)"],
             "B: back (owner .. commit + exchanges)": [
                 "gx_x1(X1 all-to-all + host)", "gx_owner(own_claim..own_finish)", "gx_x2(X2 all-to-all)",
                 "gx_decide(gx_decide + x3want)", "scan(tile/chunk_scan)", "gx_flush_fn(fn_info/fn_chain/fn_pack)",
                 "gx_allgather(flush descriptors)", "gx_alloc_scan(gx_scan_kernel)", "flush(flush_kernel)",
                 "gx_place_meta(place_kernel part 1)", "gx_x3(X3 all-to-all + host)", "gx_commit(own_commit)"],
             "B2: arena copy": ["place(place_kernel)"]}
SHA_MIX_CEILING_WI_NS = 425.0  # tools/sha_peak.hip: the SHA-1 instruction mix on register-resident data
HBM_ACHIEVABLE_GBS = 6300.0    # MI355X_MICROARCH.md HBM section: ~6.3 TB/s achievable
# kernels launched per batch in the config-2 pipeline (the rest once); setup kernels are not counted
_PIPE_SKIP = ("corpus_kernel", "__amd_rocclr", "idx_clear_kernel", "_config")
_PIPE_LAUNCHES = {"lane_repair_kernel": 2}


def pipeline_traffic(pmc):
    """Counted HBM bytes of one batch: every pipeline kernel's per-launch figure x its launches per batch
    (None without a PMC file for this workload, or for a workload with an LZ4 pass per batch)."""
    if not pmc or any(k.startswith("lz4") for k in pmc):
        return None
    tot = 0
    for k, v in pmc.items():
        if isinstance(v, dict) and "hbm_bytes_per_launch" in v and not any(k.startswith(s) for s in _PIPE_SKIP):
            tot += v["hbm_bytes_per_launch"] * _PIPE_LAUNCHES.get(k, 1)
    return tot or None


# template arguments a kernel's name carries in the PMC files (gmax2's defaulted COND is spelled out
# since round 6: "gmax2_kernel<true, false>")
PMC_SUFFIXES = ("", "<5>", "<7>", "<true>", "<false>", "<true, false>", "<false, false>")


def pmc_lookup(pmc, kern):
    """The PMC entry of kernel `kern` (any of its template instances above), or {}."""
    return next((pmc[kern + t] for t in PMC_SUFFIXES if kern + t in pmc), {})


def load_pmc(want):
    """Per-launch PMC figures of the newest committed rocprofv3 pass (scripts/r02_traffic.sh ->
    scripts/traffic.py -> profiles/*_traffic.json) taken on this same workload (`want`: the
    workload's `_config` keys; a file without "workload" was taken on config 2)."""
    import glob
    want = dict(want)
    want.setdefault("front", "two-pass")            # (a fused-front pass, §6b, is only its own workload's)
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))   # names sort by round, version
    for f in reversed(files):
        d = json.load(open(f))
        cfg = dict(d.get("_config", {}))
        cfg.setdefault("workload", "config2")
        cfg.setdefault("front", "two-pass")
        if all(cfg.get(k) == v for k, v in want.items()):
            return d, os.path.relpath(f, ROOT)
    return {}, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 20 timed steps (~1.2 s at N=1): the primed pipeline's one fill and drain per timed region are
    # spread over 320 batches instead of 80
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--blocks", type=int, default=512)
    ap.add_argument("--batch", type=int, default=0,
                    help="blocks per batch (default 32; config5 16: the step's first H2D and last drain, which "
                         "nothing overlaps, are shorter: 40.2 / 40.6 vs 38.9 / 39.5 GB/s, profiles/r04_c5_b_summary.txt, "
                         "profiles/r04_c5_c_summary.txt)")
    ap.add_argument("--block-mib", type=int, default=128)
    ap.add_argument("--seg-mib", type=int, default=1)
    ap.add_argument("--dup-ppm", type=int, default=500000)
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--index-log2", type=int, default=27)
    ap.add_argument("--hasher", type=int, default=0)
    ap.add_argument("--cpu-sample-blocks", type=int, default=0,
                    help="blocks of the CPU baseline sample (default: the first batch, checked chunk by chunk)")
    ap.add_argument("--no-cpu", action="store_true",
                    help="no CPU leg: neither the timed baseline sample nor the whole-corpus storeSize check")
    ap.add_argument("--no-corpus-check", action="store_true",
                    help="skip the whole-corpus check (every block's storeSize from the timed steps vs the oracle)")
    ap.add_argument("--serial", action="store_true",
                    help="one batch at a time (no stream overlap): clean per-kernel stage times")
    ap.add_argument("--read-blocks", type=int, default=0,
                    help="read side: blocks reduced into a separate context and rebuilt on the GPU (default 0: "
                         "off, so a rocprof summary of the default bench holds only the timed pipeline's kernels)")
    ap.add_argument("--keep-recipes", type=int, default=1,
                    help="storeDB's recipe SET per block into the device recipe store (default 1, as the reference)")
    ap.add_argument("--depth", type=int, default=0,
                    help="batches in flight (1..5, pipelined mode; default 4 for the primed config-2 line, else 3; config4 5: the LZ4 passes of two "
                         "batches overlap while the front halves of the next ones run)")
    ap.add_argument("--alone", action="store_true",
                    help="after the timed region, one untimed serial pass: per-kernel rooflines without co-running "
                         "batches (on by default for the config-2 line; --no-alone when the bench runs under a "
                         "profiler whose summary must hold only the timed pipeline's kernels)")
    ap.add_argument("--no-alone", action="store_true")
    ap.add_argument("--no-prime", action="store_true",
                    help="drain the pipeline and reset synchronously at every step (the round-4 step shape; "
                         "default: steps back to back, hdrf_reset_async; config 5 packets are never primed)")
    ap.add_argument("--arena-slots", type=int, default=0,
                    help="32 MiB container slots (4 rings); each ring must hold a batch's closed containers "
                         "(default 512; config4 1792, so a ring also holds the closes of the batches whose LZ4 "
                         "passes are still running: stream B waits only on the pass three batches back; "
                         "1792 vs 1280: 37.14 / 37.22 vs 36.96 / 36.94 GB/s, profiles/r02_c4_arena_ab.txt)")
    ap.add_argument("--packet-kib", type=int, default=0,
                    help="config5: deliver every block as packets of this many KiB (hdrf_rx_begin / "
                         "hdrf_append_packet / hdrf_submit_slot, one block per submit: the JNI shape); "
                         "0 = whole blocks through hdrf_submit_host")
    ap.add_argument("--packet-threads", type=int, default=4,
                    help="config5 packets: receiver threads appending different blocks' packets concurrently")
    ap.add_argument("--no-drain", action="store_true",
                    help="config5: ring arena without durable containers (A/B of the drain's cost only)")
    ap.add_argument("--packet-driver", choices=["python", "cpp"], default="python",
                    help="config5 packets: 'cpp' runs tests/cpp/packet_driver.cpp (native receiver threads on the "
                         "C-ABI the JNI binding calls, durable containers drained after every block) as a child "
                         "process and reports its rate")
    ap.add_argument("--compressor", type=int, choices=[0, 1, 2], default=0,
                    help="DataNode.compressor (DN/DataNode.java:438): 1 dedup, 2 dedup + Lz4Codec closed containers "
                         "(the reference's default); 0 = the workload's own (config4 2, else 1)")
    ap.add_argument("--mirror", choices=["ring", "socket", "none"], default="ring",
                    help="config5 native packets: every packet forwarded downstream before it is appended "
                         "(mirrorPacketTo, DN/BlockReceiver.java:635-641): 'ring' a byte ring drained by a consumer "
                         "thread per receiver, 'socket' an AF_UNIX stream socket, 'none' a single-replica write")
    ap.add_argument("--packet-batch", action="store_true",
                    help="config5 native packets: every receive round's blocks submitted as one batch "
                         "(hdrf_submit_slots) instead of one block per batch (hdrf_submit_slot)")
    ap.add_argument("--mixed", action="store_true",
                    help="config5: config 4's mixed-entropy corpus instead of config 2's")
    ap.add_argument("--no-sub", action="store_true",
                    help="config 2 at N=1 also runs short config-4 and config-5 lines (the reference's default "
                         "compressor 2, DN/DataNode.java:438) as child processes before its own run and carries "
                         "them under \"configs\"; this turns them off")
    ap.add_argument("--workload", choices=["config2", "config4", "config5"], default="config2",
                    help="config4: mixed-entropy blocks (random/text/binary), dedup + Lz4Codec containers; "
                         "config5: host-resident (pinned) blocks streamed H2D on a side stream (PCIe-inclusive)")
    return ap.parse_args()


PK_SAMPLE_BLOCKS = 8          # config-5 packets: blocks whose chunks and closed containers are checked
PK_SAMPLE_IDS = 16            # ... container ids kept per storer range (the sample's closes lie below)


def packet_driver_line(a):
    """config5 through the native packet driver (a child process; this process touches the GPU only
    after it, for the checks and the link probe)."""
    import shutil
    import subprocess
    import tempfile
    exe = os.path.join(ROOT, "tools", "_build", "packet_driver")
    if not os.path.exists(exe):
        import __graft_entry__ as ge
        exe = ge.build_packet_driver()
    nb = 128 if a.blocks == 512 else a.blocks
    pk = a.packet_kib or 64
    compressor = a.compressor or 1
    cmd = [exe, str(nb), str(a.block_mib), str(pk), str(a.packet_threads), str(a.steps), "--compressor",
           str(compressor), "--mirror", a.mirror, "--arena-slots", str(a.arena_slots or 512)]
    cmd += ["--batch"] * a.packet_batch + ["--mixed"] * a.mixed
    out_dir = None
    if not a.no_cpu:
        # one more, untimed step keeps its results: every block's storeSize, the sample's chunks and
        # the containers its closes wrote (bench.py checks them against the oracle below)
        out_dir = tempfile.mkdtemp(prefix="hdrf_c5pk_")
        cmd += [out_dir, "--out-blocks", str(PK_SAMPLE_BLOCKS), "--out-containers", str(PK_SAMPLE_IDS)]
    # (the child keeps HIP's default hardware queues: GPU_MAX_HW_QUEUES 4 / 8 / 6, with and without
    # per-receive-buffer H2D streams, all within the run-to-run spread, profiles/r04_c5_f_queues_ab.txt)
    env = dict(os.environ)
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=1500, env=env)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        if out_dir:
            shutil.rmtree(out_dir, ignore_errors=True)
        raise SystemExit("packet driver failed (%d): %s %s" % (r.returncode, r.stdout[-2000:], r.stderr[-2000:]))
    d = json.loads(r.stdout.strip().splitlines()[-1])
    S = a.block_mib << 20
    import torch                              # (torch initialises HIP before libhdrf does in this process)
    link = link_probe(torch, 0, S)
    check = None
    if out_dir:
        try:
            check = packet_check(out_dir, nb, a.block_mib, compressor, a.mixed)
        finally:
            shutil.rmtree(out_dir, ignore_errors=True)
    drained = d["drained_bytes_last_step"]
    line = {"metric": METRIC, "value": d["GB_s"], "unit": "GB/s", "n_gpus": 1, "steps": a.steps, "warmup": 1,
            "ms_per_step": round(nb * S / d["GB_s"] / 1e6, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic",
            "config": {"workload": "config5: %d x %d MiB host-resident (pinned) blocks, 50%% dup%s, %d KiB packets from %d "
                                   "native receiver threads, each packet mirrored downstream (%s) before "
                                   "hdrf_append_packet, %s, FIFO, compressor %d, durable containers drained after "
                                   "every batch, fresh index per step"
                                   % (nb, a.block_mib, ", mixed entropy" if a.mixed else "", pk, a.packet_threads,
                                      a.mirror, "hdrf_submit_slots (a receive round per batch)" if a.packet_batch
                                      else "hdrf_submit_slot (one block per batch)", compressor),
                       "blocks_per_gpu": nb, "block_bytes": S, "parallelism": "dp1"},
            "roofline": None, "cpu_baseline": None, "mirror": a.mirror != "none", "mirror_ok": d.get("mirror_ok"),
            "packet_driver": d, "driver_wall_s": round(wall, 2), "oracle_check": check,
            "rate_note": "value = bytes of all timed steps / their time (packet_driver.GB_s); per-step rates, their "
                         "median and the fastest step beside it (host-side receive copies: the rate moves with the "
                         "shared host's memory load, DESIGN.md §11)"}
    line["pcie"] = pcie_entry(d["GB_s"], nb * S, drained, nb * S / d["GB_s"] / 1e9, link)
    print(json.dumps(line), flush=True)


SUB_RUNS = {
    # config 4: mixed-entropy blocks, dedup + Lz4Codec on closed containers (compressor 2), depth 5;
    # the CPU leg checks the container files of its sample
    "config4": ["--workload", "config4", "--steps", "2", "--warmup", "1", "--cpu-sample-blocks", "8"],
    # config 5: host-resident whole blocks under the reference default (compressor 2), every container
    # file drained D2H after each completed batch, PCIe-inclusive
    "config5": ["--workload", "config5", "--compressor", "2", "--steps", "2", "--warmup", "1",
                "--cpu-sample-blocks", "8"],
    # config 5 as worded (the JNI's packet path): 64 KiB packets from 4 native receiver threads, each
    # mirrored downstream before hdrf_append_packet (DN/BlockReceiver.java:634-658, 877-896), every
    # receive round submitted as one batch (hdrf_submit_slots, the JNI's submitSlots0), compressor 2,
    # durable containers drained after every batch
    "config5_packets": ["--workload", "config5", "--packet-driver", "cpp", "--packet-batch", "--compressor", "2",
                        "--mirror", "ring", "--steps", "5"],
}


def packet_check(out_dir, nb, block_mib, compressor, mixed):
    """The packet driver's kept step against the oracle: every block's storeSize (store-size mode over
    the whole corpus), the first PK_SAMPLE_BLOCKS blocks chunk for chunk (END offsets, digests,
    is_new), and every container the oracle closes within them (raw, or the Lz4Codec file under
    compressor 2, DN/DataDeduplicator.java:748-818) byte for byte with the drained file."""
    import numpy as np
    from hdrf_amd.corpus import corpus_roots
    from hdrf_amd.lib import Context
    from oracle.oracle import Oracle
    S, seg = block_mib << 20, 1 << 20
    spb = S // seg
    got = np.loadtxt(os.path.join(out_dir, "blocks.txt"), dtype=np.int64).reshape(-1, 3)
    raw = open(os.path.join(out_dir, "containers.bin"), "rb").read()
    disk, o = {}, 0
    while o < len(raw):
        cid, closed = np.frombuffer(raw, np.uint32, 2, o)
        n = int(np.frombuffer(raw, np.uint64, 1, o + 8)[0])
        disk[int(cid)] = (raw[o + 16:o + 16 + n], bool(closed))
        o += 16 + n
    # the same corpus the driver generated (hdrf_corpus_fill_kind, seed 20251015, 50 % dup)
    G = 16
    ctx = Context(max_block_bytes=S, max_batch_blocks=1, index_log2=10, arena_slots=8)
    dev = ctx.dev_alloc(nb * S)
    ctx.corpus_fill(dev, corpus_roots(20251015, 500000, nb, spb), nb, spb, seg, 20251015, mixed=mixed)
    host = ctx.host_alloc(G * S)
    lean = Oracle(compressor=compressor, store_only=True)
    full = Oracle(compressor=compressor)
    nthr = max(1, cpu_share() - 1)
    ss, chunk_bad, nchunks = [], 0, 0
    for b0 in range(0, nb, G):
        k = min(G, nb - b0)
        ctx.L.hdrf_memcpy_d2h(ctx._h, host.ctypes.data, dev + b0 * S, k * S)
        blks = [host[i * S:(i + 1) * S] for i in range(k)]
        ss.extend(int(x) for x in lean.reduce_many(blks, list(range(b0, b0 + k)), nthr))
        if b0 < PK_SAMPLE_BLOCKS:
            m = min(k, PK_SAMPLE_BLOCKS - b0)
            for i, e in enumerate(full.reduce_many_full(blks[:m], list(range(b0, b0 + m)), nthr)):
                n = len(e["offsets"])
                f = open(os.path.join(out_dir, "blk_%d.bin" % (b0 + i)), "rb").read()
                H = e["digests"].shape[1]
                ok = (len(f) == n * (5 + H) and np.array_equal(np.frombuffer(f, np.uint32, n, 0), e["offsets"])
                      and np.array_equal(np.frombuffer(f, np.uint8, n * H, 4 * n).reshape(n, H), e["digests"])
                      and np.array_equal(np.frombuffer(f, np.uint8, n, (4 + H) * n), e["is_new"]))
                chunk_bad += not ok
                nchunks += n
    ctx.host_free(host)
    ctx.dev_free(dev)
    ctx.close()
    alloc = full.allocator()
    checked = bad = 0
    for t in range(3):
        for cid in range(t << 22, int.from_bytes(alloc[3 * t:3 * t + 3], "big") + 1):
            od, oc = full.container(cid)
            if od is None or not oc:
                continue                          # open after the sample: later blocks append to it
            checked += 1
            bad += int(disk.get(cid) != (od, True))
    ss = np.array(ss, np.int64)
    return {"blocks": nb, "store_size_mismatches": int((ss != got[:, 2]).sum()),
            "dedup_ratio_oracle": round(nb * S / max(int(ss.sum()), 1), 6),
            "dedup_ratio_driver": round(nb * S / max(int(got[:, 2].sum()), 1), 6),
            "sample_blocks": PK_SAMPLE_BLOCKS, "sample_chunks": nchunks, "sample_block_mismatches": chunk_bad,
            "containers_checked": checked, "container_file_mismatches": bad,
            "what": "the driver's untimed results step (same corpus, fresh index): storeSize of every block vs the "
                    "oracle in store-size mode; chunks of the first %d blocks and the containers the oracle closes "
                    "within them vs the drained chunkDir files" % PK_SAMPLE_BLOCKS}


def sub_configs():
    """The short config-4 / config-5 lines, each in a child process (run before this process touches
    the GPU, so each child has the whole card): {name: its JSON line without the per-stage table}."""
    import subprocess
    out = {}
    for name, args in SUB_RUNS.items():
        t0 = time.perf_counter()
        try:
            r = subprocess.run([sys.executable, os.path.abspath(__file__)] + args + ["--no-sub"], capture_output=True,
                               text=True, timeout=420, env=dict(os.environ))
            lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
            if r.returncode != 0 or not lines:
                out[name] = {"error": "rc %d: %s" % (r.returncode, (r.stderr or r.stdout)[-600:])}
                continue
            d = json.loads(lines[-1])
        except Exception as e:                       # a failed sub-line never voids the headline
            out[name] = {"error": repr(e)[:600]}
            continue
        d.pop("stages", None)
        if isinstance(d.get("roofline"), dict):
            d["roofline"].pop("alone", None)
        d["command"] = "python bench.py " + " ".join(args)
        d["wall_s"] = round(time.perf_counter() - t0, 1)
        out[name] = d
        print("sub-line %s: %.3f %s (%.0f s)" % (name, d.get("value") or 0, d.get("unit"), d["wall_s"]),
              file=sys.stderr, flush=True)
    return out


def pcie_entry(value, h2d_bytes, d2h_bytes, step_s, link):
    """The link figures of a config-5 line: the raw probes and what the step moved over PCIe."""
    moved = (h2d_bytes + d2h_bytes) / step_s / 1e9
    return {"h2d_GB_s_raw_copy": round(link["h2d"], 2), "d2h_GB_s_raw_copy": round(link["d2h"], 2),
            "bidirectional_GB_s_raw_copy": round(link["bidir"], 2),
            "bidirectional_split_GB_s": {"h2d": round(link["bidir_h2d"], 2), "d2h": round(link["bidir_d2h"], 2)},
            "value_over_raw_copy": round(value / link["h2d"], 4),
            "value_over_bidirectional_raw": round(value / link["bidir_h2d"], 4),
            "link_GB_s": round(moved, 2), "link_frac_of_bidirectional_raw": round(moved / link["bidir"], 4),
            "drained_container_bytes_per_step": int(d2h_bytes),
            "d2h_GB_s_drain": round(d2h_bytes / step_s / 1e9, 2),
            "raw_copy": "pinned host <-> HBM, 128 MiB hipMemcpyAsync pieces, 4 in flight per stream, timed with HIP "
                        "events (torch); bidirectional: H2D and D2H streams at once; best of %d passes (median "
                        "beside)" % link["passes"],
            "raw_copy_median_GB_s": link["median"], "bidirectional_passes_GB_s": link["bidir_passes_GB_s"],
            "value_over_bidirectional_raw_def": "value / the H2D rate the link sustains while D2H runs at once",
            "note": "value is PCIe-inclusive: host buffers -> HBM -> reduced, and every container file "
                    "(retain_containers, the JNI binding's mode) drained D2H to pinned host memory after each "
                    "completed batch, inside the timed region"}


def main():
    a = parse()
    if a.workload == "config5" and a.packet_driver == "cpp":
        return packet_driver_line(a)
    if not a.depth:
        # config 2: depth 3 984 -> 1004 GB/s (three A/B pairs, scripts/ab_d23.txt): chunking of batch
        # k+2 starts while batch k+1 hashes instead of after batch k's read-back; round 5, primed steps:
        # depth 4 1071-1103 (mean 1093) vs depth 3 1065-1102 (mean 1084) over three A/B files
        primed_c2 = a.workload == "config2" and a.gpus == 1 and not a.no_prime and not a.serial
        a.depth = 5 if a.workload == "config4" else 4 if primed_c2 else 3
    if not a.arena_slots:
        # config 5 keeps durable containers: a submit is refused while the worst-case closes of the
        # batches in flight (<= 2 x new bytes / maxSize + 1 per block and storer range, three 32-block
        # batches) could reach an undrained slot, so its rings hold ~500 slots each (64 GiB of 288)
        a.arena_slots = {"config4": 1792, "config5": 2048}.get(a.workload, 512)
    # the batch pipeline uses five streams (chunking, SHA, index, store, recipe copies) and config 4
    # two more LZ4 streams: hardware queues for all of them (HIP's default is 4, and streams sharing
    # a queue serialise); read when HIP initialises
    os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    subs = None
    if world == 1 and a.workload == "config2" and not a.no_sub and not a.serial:
        subs = sub_configs()                             # before this process initialises the GPU
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist
        if os.environ.get("HDRF_BENCH_SAME_DEVICE") == "1":
            local = 0
            dist.init_process_group(backend="gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))

    from hdrf_amd.corpus import corpus_roots
    from hdrf_amd.lib import STAGES, Context

    S = a.block_mib << 20
    seg = a.seg_mib << 20
    spb = S // seg
    if not a.batch:
        a.batch = 16 if a.workload == "config5" else 32
    nb, B = a.blocks, min(a.batch, a.blocks)
    if nb % B:
        raise SystemExit("--blocks must be a multiple of --batch")
    # One node, one index: at N > 1 the GPUs are ranks of ONE reduction over the global block
    # sequence (hdrf_amd/node.py): a global corpus of world*nb blocks, every global batch takes B
    # blocks from each rank (rank-major), the index is partitioned by digest prefix.
    host = a.workload == "config5"
    mixed = a.workload == "config4" or (host and a.mixed)
    if (mixed or host) and world > 1:
        raise SystemExit("config4/config5 run on single-node contexts only")
    if host and a.blocks == 512:
        nb = 128                                         # 16 GiB of pinned host memory
    compressor = a.compressor or (2 if mixed else 1)
    # config 5 is the DataNode write path: durable containers (retain_containers, as the JNI binding
    # opens it) handed out to pinned host memory after every completed batch, inside the timed region
    ctx = Context(device=local, hasher=a.hasher, max_block_bytes=S, max_batch_blocks=B, index_log2=a.index_log2,
                  arena_slots=a.arena_slots, keep_recipes=a.keep_recipes, timing=1, n_ranks=world, rank=rank,
                  compressor=compressor, retain_containers=1 if host and not a.no_drain else 0)
    node = None
    if world > 1:
        from hdrf_amd.node import NodeRank, global_block
        node = NodeRank(ctx)
    seed = a.seed
    groots = corpus_roots(seed, a.dup_ppm, nb * world, spb).reshape(nb * world, spb)
    if world > 1:
        mine = [global_block(L, rank, world, B) for L in range(nb)]
        roots = groots[mine].reshape(-1)
    else:
        roots = groots.reshape(-1)
    total = nb * S + 4096
    dev = ctx.dev_alloc(total)
    ctx.corpus_fill(dev, roots, nb, spb, seg, seed, mixed=mixed)
    hbuf, link, dbuf = None, None, None
    drained = {"events": 0, "bytes": 0}
    if host:                                             # the DataNode's received blocks, in host memory
        hbuf = ctx.host_alloc(nb * S)
        ctx.L.hdrf_memcpy_d2h(ctx._h, hbuf.ctypes.data, dev, nb * S)
        dbuf = None if a.no_drain else ctx.host_alloc(1 << 30)   # the drained container files (pinned)
        link = link_probe(torch, local, S)
    batches = []
    for b0 in range(0, nb, B):
        k = min(B, nb - b0)
        batches.append(([dev + (b0 + i) * S for i in range(k)], [S] * k,
                        [total - (b0 + i) * S for i in range(k)], [b0 + i for i in range(k)]))

    n_chunks = np.zeros(nb, np.int64)
    store = np.zeros(nb, np.int64)

    def drain():
        if dbuf is not None:
            e, n = ctx.drain_into(dbuf.ctypes.data, dbuf.size)
            drained["events"] += e
            drained["bytes"] += n

    def step():
        if node is None:
            ctx.reset()                                  # a fresh DataNode index each step
        else:
            node.reset()
        j = 0

        def collect():
            nonlocal j
            for i in range(ctx.last_nblocks()):
                n_chunks[j], store[j] = ctx.batch_info(i)
                j += 1

        if node is None and a.serial:
            for ptrs, lens, rd, ids in batches:
                ctx.reduce_batch(ptrs, lens, rd, ids)
                collect()
        elif host and a.packet_kib:
            # packet-granular receive, one block per submit (the JNI shape): each block's packets are
            # appended as they "arrive" (chunk H2D on the copy stream) while earlier blocks reduce;
            # T receiver threads (one per block, as DataXceiver threads) append concurrently
            import threading
            P, T = a.packet_kib << 10, max(1, a.packet_threads)
            pend = 0

            def receive(rx, b):
                base = hbuf.ctypes.data + b * S
                for o in range(0, S, P):
                    ctx.append_packet(rx, base + o, min(P, S - o))

            for g in range(0, nb, T):
                grp = list(range(g, min(nb, g + T)))
                while pend + len(grp) > 8 or pend >= 5:          # 8 receive buffers, depth 5
                    ctx.wait_batch()
                    collect()
                    pend -= 1
                rxs = [ctx.rx_begin(b) for b in grp]
                th = [threading.Thread(target=receive, args=(rx, b)) for rx, b in zip(rxs, grp)]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
                for rx in rxs:                             # submitted in arrival (block) order
                    if pend >= 5:
                        ctx.wait_batch()
                        collect()
                        drain()
                        pend -= 1
                    ctx.submit_slot(rx)
                    pend += 1
            for _ in range(pend):
                ctx.wait_batch()
                collect()
                drain()
        elif host:
            # streaming: the H2D copies of batch k+1 (side stream) overlap the reduction of batch k;
            # after each completed batch its containers go D2H (stream D) while later batches run
            for k, (ptrs, lens, rd, ids) in enumerate(batches):
                ctx.submit_host([hbuf.ctypes.data + (p - dev) for p in ptrs], lens, ids)
                if k >= 2:
                    ctx.wait_batch()
                    collect()
                    drain()
            for _ in range(min(2, len(batches))):
                ctx.wait_batch()
                collect()
                drain()
        elif node is None:
            # pipelined: chunking of batch k+2, SHA of batch k+1 and index/store of batch k overlap
            depth = a.depth
            for k, (ptrs, lens, rd, ids) in enumerate(batches):
                ctx.submit_batch(ptrs, lens, rd, ids)
                if k >= depth - 1:
                    ctx.wait_batch()
                    collect()
            for _ in range(min(depth - 1, len(batches))):
                ctx.wait_batch()
                collect()
        elif a.serial:
            for ptrs, lens, rd, ids in batches:
                node.reduce_batch(ptrs, lens, rd, ids, rank * B)
                collect()
        else:
            # pipelined: the front half of global batch k+1 overlaps batch k's exchanges + store
            node.reduce_batches([(ptrs, lens, rd, ids, rank * B) for ptrs, lens, rd, ids in batches],
                                lambda k: collect())

    def barrier():
        if dist is not None:
            dist.barrier()

    # Config 2 (device-resident, one context): the steps run back to back with the pipeline kept
    # primed, as a continuously written DataNode's would be.  Each step is still one fresh DataNode
    # reducing the whole corpus (hdrf_reset_async: the next batch starts a new index generation while
    # the previous step's last batches complete), and every batch's results are collected inside the
    # timed region; only the per-step pipeline fill and drain (an empty front or back stream for about
    # one batch chain per step) are gone.  --no-prime: the round-4 shape (drain + reset per step).
    # Config 5 whole blocks (durable containers) too: each step's containers are drained as its
    # batches complete, the next step's H2D copies start beside the last batches and drains.
    primed = not a.serial and not a.no_prime and not (host and a.packet_kib)

    def run_primed_node(nsteps):
        # N > 1: every step's batches in one pipelined sequence, hdrf_reset_async on every rank before
        # the first front of each step (hdrf_amd/node.py reduce_batches gens), so the previous step's
        # last batches complete while the next step's fronts run — the N = 1 step shape
        nbatch = len(batches)
        seq = [(ptrs, lens, rd, ids, rank * B) for _ in range(nsteps) for ptrs, lens, rd, ids in batches]

        def done(k):
            k0 = (k % nbatch) * B
            for i in range(ctx.last_nblocks()):
                n_chunks[k0 + i], store[k0 + i] = ctx.batch_info(i)

        node.reduce_batches(seq, done, gens=[s * nbatch for s in range(nsteps)])

    def run_primed(nsteps):
        if node is not None:
            return run_primed_node(nsteps)
        from collections import deque
        q = deque()

        def collect_one():
            k0 = q.popleft()
            ctx.wait_batch()
            for i in range(ctx.last_nblocks()):
                n_chunks[k0 + i], store[k0 + i] = ctx.batch_info(i)

        for _ in range(nsteps):
            ctx.reset_async()
            for k, (ptrs, lens, rd, ids) in enumerate(batches):
                if host:
                    # config 5: the streaming shape of step() (H2D of batch k+1 beside the reduction of
                    # k, containers drained after every completed batch), steps back to back: the
                    # next step's first copies run beside this step's last batches and drains
                    ctx.submit_host([hbuf.ctypes.data + (p - dev) for p in ptrs], lens, ids)
                    q.append(k * B)
                    if len(q) >= 3:
                        collect_one()
                        drain()
                    continue
                if len(q) >= a.depth:
                    collect_one()
                ctx.submit_batch(ptrs, lens, rd, ids)
                q.append(k * B)
        while q:
            collect_one()
            drain()

    if primed:
        run_primed(a.warmup)
    else:
        for _ in range(a.warmup):
            step()
    drained.update(events=0, bytes=0)
    ctx.stage_times(reset=True)
    # HDRF_LZ4_PHASES=1 with the profiling build (-DHDRF_LZ4_PROF, scripts/r05_lzp_c4.sh): the LZ4
    # parse's per-phase shader clocks over the timed steps, inside the pipeline
    lzp_lib = getattr(ctx.L, "hdrf_debug_lz4_prof", None) if os.environ.get("HDRF_LZ4_PHASES") else None
    lzp_buf = None
    if lzp_lib is not None:
        import ctypes
        lzp_lib.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        lzp_buf = (ctypes.c_ulonglong * 16)()
        ctx.synchronize()
        lzp_lib(lzp_buf, 1)
    if node is not None:
        node.phase_ms = {}
    barrier()
    torch.cuda.synchronize()
    ctx.synchronize()
    t0 = time.perf_counter()
    if primed:
        run_primed(a.steps)
    else:
        for _ in range(a.steps):
            step()
    ctx.synchronize()
    torch.cuda.synchronize()
    barrier()
    el = time.perf_counter() - t0
    stage_ms = ctx.stage_times(reset=True)
    lz4_phases = None
    if lzp_buf is not None:
        lzp_lib(lzp_buf, 1)
        v = list(lzp_buf)
        tot = sum(v[:8])
        nbat, nfound, nchain = v[8], v[9], v[10]
        names = ["search batch", "catch-up+literals", "chain top+extension", "tokens+table", "Cw load+compare",
                 "-", "last literals", "-"]
        per_ev = [nbat, nfound, nfound + nchain, nfound + nchain, nfound + nchain, 1, 1, 1]
        lz4_phases = {"cycles_per_sequence": round(tot / max(1, nfound + nchain), 1),
                      "search_batches": nbat, "found": nfound, "chained": nchain,
                      "phases": {names[i]: {"share": round(v[i] / max(1, tot), 4),
                                            "cyc_per_event": round(v[i] / max(1, per_ev[i]), 1)}
                                 for i in range(8) if v[i]}}
    alone_ms = None
    alone = (a.alone or (a.workload == "config2" and not a.no_alone)) and not a.no_alone
    if alone and node is None and not a.serial and not host:
        # one extra, untimed serial pass (one batch at a time): the same kernels without the
        # co-running batch, for the per-kernel "alone" rooflines next to the in-pipeline ones
        ctx.reset()
        for ptrs, lens, rd, ids in batches:
            ctx.reduce_batch(ptrs, lens, rd, ids)
        alone_ms = ctx.stage_times(reset=True)
    if dist is not None:
        t = torch.tensor([el], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms_step = el / a.steps * 1e3
    logical = nb * S * world
    value = logical / (el / a.steps) / 1e9

    # ---- rooflines (algorithmic bytes / HIP-event time on the library's streams) ---------------
    nbatch = len(batches)
    chunks_step = int(n_chunks.sum())
    new_bytes = int(store.sum())
    S_batch = nb * S / nbatch
    per_launch = {   # algorithmic HBM bytes per launch
        "gmax(gmax_kernel)": S_batch * (1 + 1 / 16),                      # read block bytes, write granule maxima
        "walk(lane_walk_kernel)": (S_batch + (4 + 4 * (5 if a.hasher == 0 else 7)) * chunks_step / nbatch if FUSED
                                   else S_batch / 16 + 4 * chunks_step / nbatch),  # fused: bytes in, cuts + digests out;
                                                                                   # walk: read maxima, write cuts
        STAGES[2]: S_batch + 40 * chunks_step / nbatch,                   # read chunk bytes + offsets, write mid-state
        STAGES[9]: (2 * new_bytes + 16 * chunks_step) / nbatch,           # read+write new bytes, chunk metadata
    }
    avg = {name: ms / a.steps / nbatch for name, ms in zip(STAGES, stage_ms)}
    stages = {}
    for name, ms in zip(STAGES, stage_ms):
        d = {"ms_per_step": round(ms / a.steps, 3), "avg_launch_ms": round(avg[name], 4)}
        if name in per_launch and avg[name] > 0:
            d["GB_s"] = round(per_launch[name] / (avg[name] * 1e-3) / 1e9, 1)
        stages[name] = d
    pmc, pmc_src = load_pmc({"blocks": nb, "block_mib": a.block_mib, "batch": B, "n_gpus": world,
                             "hasher": a.hasher, "workload": a.workload, "front": "fused" if FUSED else "two-pass"})
    sha_k = KERNEL_OF[STAGES[2]] + ("<5>" if a.hasher == 0 else "<7>")

    def hbm_entry(name):
        ms = avg[name]
        ach = per_launch[name] / (ms * 1e-3) / 1e9 if ms > 0 else 0.0
        return {"bound": "hbm", "kernel": KERNEL_OF[name], "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4), "avg_launch_ms": round(ms, 4),
                "algorithmic_bytes_per_launch": int(per_launch[name]),
                "traffic": pmc_lookup(pmc, KERNEL_OF[name]).get("hbm_bytes_per_launch")}

    # per-stream chains: the batch period is set by the longest one (the critical path)
    chain_def = CHAINS_GX if world > 1 else CHAINS
    chains = {c: round(sum(avg[s] for s in st), 4) for c, st in chain_def.items()}
    crit = max(chains, key=chains.get)
    chunk_ms = chains["W: chunking"]
    chunking = {"kernels": ("lane_hash (cuts and SHA in one pass over the bytes) + stitch (one batch, in pipeline)"
                            if FUSED else "gmax + lane walk + stitch (one batch, in pipeline)"), "avg_batch_ms": chunk_ms,
                "achieved": round(S_batch / (chunk_ms * 1e-3) / 1e9, 1) if chunk_ms > 0 else None,
                "peak": HBM_PEAK_GBS, "unit": "GB/s (block bytes chunked)",
                "frac": round(S_batch / (chunk_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if chunk_ms > 0 else None,
                "gmax": hbm_entry("gmax(gmax_kernel)"), "walk": hbm_entry("walk(lane_walk_kernel)")}
    sha = hbm_entry(STAGES[2])
    sha_prof = pmc.get(sha_k, {})
    if sha_prof.get("sq_insts_valu") and avg[STAGES[2]] > 0:
        # SHA is integer-VALU bound: wave-instructions per launch (PMC SQ_INSTS_VALU) over the
        # measured launch time, against the full-rate v_add_u32 peak (profiles/r01_valu_peak.txt)
        # and the SHA-1 instruction mix's own ceiling (tools/sha_peak.hip)
        wi_ns = sha_prof["sq_insts_valu"] / (avg[STAGES[2]] * 1e6)
        sha["limiter"] = "int-VALU"
        sha["valu"] = {"wave_instr_per_ns": round(wi_ns, 1), "peak": VALU_PEAK_WI_NS,
                       "frac": round(wi_ns / VALU_PEAK_WI_NS, 4), "mix_ceiling": SHA_MIX_CEILING_WI_NS,
                       "frac_of_mix_ceiling": round(wi_ns / SHA_MIX_CEILING_WI_NS, 4),
                       "sq_insts_valu_per_launch": int(sha_prof["sq_insts_valu"])}
    place = hbm_entry(STAGES[9])
    lz4 = None
    if compressor == 2:
        # the LZ4 pass per batch: closed containers read + Lz4Codec files written, over the stage's
        # average time from the place kernel's end to the pack kernel's end on its LZ4 stream (two
        # batches' passes overlap, so this is a latency, not an exclusive share of the GPU)
        st = ctx.stats()
        lz_ms = avg["compress(lz4_seg/lz4_pack)"]
        lz_bytes = (st["closed_raw_bytes"] + st["closed_file_bytes"]) / max(1, nbatch)   # stats: since the last reset = one step
        ach = lz_bytes / (lz_ms * 1e-3) / 1e9 if lz_ms > 0 else 0.0
        lz4 = {"bound": "hbm", "kernel": "lz4_seg_kernel", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
               "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 5), "avg_launch_ms": round(lz_ms, 4),
               "algorithmic_bytes_per_launch": int(lz_bytes),
               "traffic": pmc.get("lz4_seg_kernel<false>", {}).get("hbm_bytes_per_launch"),
               "limiter": "latency of the greedy parse's per-sequence dependent chain (one wave per 261,100-B "
                          "segment; the 10 KiB tagged LDS table allows 16 waves/CU; 99 VGPRs; VALU issue 0.093 and "
                          "SALU 0.125 per SIMD-cycle, half of wave time at s_waitcnt on the table round trip and the "
                          "candidate load); profiles/r05_lz4_pmc.txt, profiles/r05_lz4_phases_c4.txt"}
    # the line's roofline: the dominant kernel of the critical chain
    if FUSED:
        # the fused pass is the front: block bytes read once; int-VALU the other bound (SHA-1's mix)
        fz = chunking["walk"]
        fz_prof = next((pmc[k] for k in ("lane_hash_kernel<5>", "lane_hash_kernel<7>") if k in pmc), {})
        if fz_prof.get("sq_insts_valu") and avg["walk(lane_walk_kernel)"] > 0:
            wi_ns = fz_prof["sq_insts_valu"] / (avg["walk(lane_walk_kernel)"] * 1e6)
            fz["valu"] = {"wave_instr_per_ns": round(wi_ns, 1), "peak": VALU_PEAK_WI_NS,
                          "frac": round(wi_ns / VALU_PEAK_WI_NS, 4), "mix_ceiling": SHA_MIX_CEILING_WI_NS,
                          "frac_of_mix_ceiling": round(wi_ns / SHA_MIX_CEILING_WI_NS, 4),
                          "sq_insts_valu_per_launch": int(fz_prof["sq_insts_valu"])}
    top = {"W: chunking": chunking["walk"] if FUSED else chunking["gmax"], "A: SHA": sha, "B: index+store": place, "B2: store": place,
           "B: index": place, "L: LZ4": lz4, "B2: arena copy": place}.get(crit)
    if top is None:
        # a node-global chain without an HBM-bound kernel of its own (local aggregation; the back
        # phases, whose time is index atomics and the exchanges): the line names the dominant HBM kernel
        # of the rank's pipeline, place, and says which chain set the period
        top = dict(place)
        top["note"] = "critical chain %s has no HBM-streaming kernel; the entry is place_kernel's" % crit
    roofline = dict(top)
    if world > 1:
        roofline["front_period_ms"] = round(max(chains[c] for c in ("W: chunking", "A: SHA", "X: local aggregation")), 4)
        roofline["front_period_note"] = ("per-rank front half (chunking | SHA | local aggregation on three streams, "
                                         "batches overlapped): the longest of the three chains per batch")
    roofline.update({"traffic_source": pmc_src, "critical_path": crit, "chains_ms_per_batch": chains,
                     "batch_period_ms": round(el / a.steps / nbatch * 1e3, 4),
                     "chunking": chunking, "sha": sha, "place": place})
    pipe = pipeline_traffic(pmc)
    if pipe and world == 1:
        # the whole pipeline against the fabric: every kernel's counted HBM bytes per batch (PMC, the same
        # workload) over the measured batch period, beside the guide's achievable rate
        period_s = el / a.steps / nbatch
        roofline["pipeline"] = {"counted_bytes_per_batch": int(pipe), "counted_bytes_per_logical_byte":
                                round(pipe / S_batch, 3), "achieved": round(pipe / period_s / 1e9, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(pipe / period_s / 1e9 / HBM_PEAK_GBS, 4),
                                "frac_of_achievable": round(pipe / period_s / 1e9 / HBM_ACHIEVABLE_GBS, 4),
                                "achievable": HBM_ACHIEVABLE_GBS,
                                "what": "sum over the batch's kernels of 2 x FETCH_SIZE + WRITE_SIZE per launch x launches "
                                        "per batch, divided by the batch period of this run"}
    if lz4:
        roofline["lz4"] = lz4
        if lz4_phases:
            lz4["phases_in_pipeline"] = lz4_phases
    if alone_ms is not None:
        # per-kernel figures of the untimed serial pass (not part of `value`)
        ra = {}
        for name in per_launch:
            ms = alone_ms[STAGES.index(name)] / nbatch
            if ms > 0:
                ach = per_launch[name] / (ms * 1e-3) / 1e9
                ra[name] = {"avg_launch_ms": round(ms, 4), "achieved_GB_s": round(ach, 1),
                            "frac_hbm": round(ach / HBM_PEAK_GBS, 4)}
        if ra.get(STAGES[2]) and sha_prof.get("sq_insts_valu"):
            ra[STAGES[2]]["valu_frac"] = round(sha_prof["sq_insts_valu"] / (ra[STAGES[2]]["avg_launch_ms"] * 1e6)
                                              / VALU_PEAK_WI_NS, 4)
        w_alone = sum(alone_ms[STAGES.index(x)] for x in CHAINS["W: chunking"]) / nbatch
        if w_alone > 0:
            ach = S_batch / (w_alone * 1e-3) / 1e9
            ra["chunking(gmax+walk+stitch)"] = {"avg_batch_ms": round(w_alone, 4), "achieved_GB_s": round(ach, 1),
                                                "frac_hbm": round(ach / HBM_PEAK_GBS, 4)}
        roofline["alone"] = ra
        roofline["alone_note"] = ("same kernels in one untimed serial pass (one batch at a time); the "
                                  "in-pipeline figures above include co-running batches")

    node_new, node_chunks = new_bytes, chunks_step
    if dist is not None:
        t = torch.tensor([new_bytes, chunks_step], dtype=torch.int64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t)
        node_new, node_chunks = int(t[0].item()), int(t[1].item())
    dedup = {"logical_bytes": nb * S * world, "stored_bytes": node_new,
             "dedup_ratio": round(nb * S * world / max(node_new, 1), 6),
             "dup_fraction": round(1 - node_new / (nb * S * world), 6), "target_dup_fraction": a.dup_ppm / 1e6,
             "chunks": node_chunks, "mean_chunk_bytes": round(nb * S * world / max(node_chunks, 1), 1),
             "index": "one node-global index over %d GPU(s), partitioned by digest prefix" % world}

    compression = None
    if compressor == 2:
        st = ctx.stats()
        stored = st["closed_file_bytes"] + st["open_bytes"]
        compression = {"closed_containers": st["closed_containers"], "closed_raw_bytes": st["closed_raw_bytes"],
                       "closed_file_bytes": st["closed_file_bytes"], "open_raw_bytes": st["open_bytes"],
                       "lz4_ratio_closed": round(st["closed_raw_bytes"] / max(st["closed_file_bytes"], 1), 6),
                       "node_ratio": round(st["logical_bytes"] / max(stored, 1), 6),
                       "node_ratio_def": "logical / (closed Lz4Codec files + open raw containers)"}
        # SURVEY §8(d)'s config-4 ratio also counts the metadata the reference keeps in Redis: the
        # recipes (BE32 size + digests per block) and one index entry (digest key + 11-B value) per
        # distinct chunk
        meta = st["recipe_bytes"] + ctx.index_count() * (ctx.H + 11)
        compression.update({"recipe_bytes": st["recipe_bytes"], "index_bytes": meta - st["recipe_bytes"],
                            "node_ratio_with_metadata": round(st["logical_bytes"] / max(stored + meta, 1), 6)})
    read_side = None
    if rank == 0 and world == 1 and a.read_blocks > 0 and not host:
        read_side = read_bench(ctx, dev, S, min(a.read_blocks, nb), a.hasher, compressor)
    cpu = None
    m_cpu = min(a.cpu_sample_blocks or B, nb)
    if rank == 0 and world == 1 and not a.no_cpu and m_cpu > 0:
        # the GPU's per-chunk results for the sample (one untimed pass from a fresh index, the same
        # batches as the timed steps), checked chunk by chunk against the all-cores oracle run
        ctx.reset()
        gpu_res, done = [], 0
        for ptrs, lens, rd, ids in batches:
            if done >= m_cpu:
                break
            ctx.reduce_batch(ptrs, lens, rd, ids)
            for i in range(ctx.last_nblocks()):
                if done < m_cpu:
                    gpu_res.append(ctx.batch_result(i))
                    done += 1
        cpu = cpu_baseline(ctx, dev, S, m_cpu, store, a.hasher, compressor, gpu_res)

    if rank == 0 and world == 1 and not a.no_cpu and not a.no_corpus_check:
        # the metric's "bit-exact dedup ratio" over the WHOLE corpus: every block's storeSize from the
        # last timed step against the oracle in store-size mode, one batch at a time
        dedup["oracle_check"] = corpus_check(ctx, dev, S, nb, B, store, a.hasher, compressor,
                                             hbuf if host else None)

    if rank == 0:
        line = {"metric": METRIC, "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": a.steps,
                "warmup": a.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True, "scaling": "weak",
                "vs_baseline": None, "dtype": "u8", "data": "synthetic",
                "config": {"workload": "config%d: %d x %d MiB %sblocks per GPU, %d%% dup (%d MiB segments), "
                                       "chunk+SHA-%s+%s index+container store%s%s, fresh index per step"
                                       % (4 if mixed else (2 if world == 1 else 3), nb, a.block_mib,
                                          "mixed-entropy (random/text/binary) " if mixed else "",
                                          a.dup_ppm // 10000, a.seg_mib, "1" if a.hasher == 0 else "224",
                                          "local" if world == 1 else "node-global (RCCL all-to-all)",
                                          " + Lz4Codec on closed containers" if compressor == 2 else "",
                                          " + recipes (device store)" if a.keep_recipes else ", no recipes"),
                           "blocks_per_gpu": nb, "block_bytes": S, "batch_blocks_per_gpu": B,
                           "batches_in_flight": node.depth if node is not None else a.depth, "steps_back_to_back": bool(primed),
                           "parallelism": "dp%d: blocks sharded by rank; one index partitioned by digest prefix"
                                          % world},
                "roofline": roofline, "cpu_baseline": cpu, "dedup": dedup, "stages": stages}
        if compression:
            line["compression"] = compression
        if subs:
            line["configs"] = subs
        if read_side:
            line["read_side"] = read_side
        if host:
            line["config"]["workload"] = ("config5: %d x %d MiB host-resident (pinned) blocks, %d%% dup%s, streamed "
                                          "H2D on a side stream overlapped with the reduction (%s), "
                                          "chunk+SHA-1+local index+container store%s, durable containers drained "
                                          "after every batch, fresh index per step"
                                          % (nb, a.block_mib, a.dup_ppm // 10000, ", mixed entropy" if mixed else "",
                                             ("%d KiB packets, %d receiver threads, hdrf_append_packet + hdrf_submit_slot, "
                                              "one block per submit" % (a.packet_kib, a.packet_threads)) if a.packet_kib else
                                             "whole blocks, hdrf_submit_host",
                                             " + Lz4Codec on closed containers" if compressor == 2 else ""))
            line["pcie"] = pcie_entry(value, nb * S, drained["bytes"] / max(1, a.steps), el / a.steps, link)
            line["pcie"]["drained_events_per_step"] = drained["events"] // max(1, a.steps)
            line["config"]["compressor"] = compressor
        if node is not None and node.phase_ms.get("batches"):
            nbt = node.phase_ms["batches"]
            line["node_back_ms_per_batch"] = {k: round(v / nbt, 3) for k, v in node.phase_ms.items() if k != "batches"}
            line["node_back_ms_per_batch"]["note"] = "rank 0 host wall time per back phase (allocator: scan, no chain)"
        print(json.dumps(line), flush=True)
    ctx.dev_free(dev)
    if hbuf is not None:
        ctx.host_free(hbuf)
        if dbuf is not None:
            ctx.host_free(dbuf)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


PASSES = 5


def link_probe(torch, device, piece):
    """The bare link: pinned host -> HBM (H2D), HBM -> pinned host (D2H), and both at once on two
    streams, in `piece`-byte async copies, 4 in flight per stream (the shape of the library's own
    copies), 8 GiB per direction and pass, timed with HIP events, best and median of PASSES passes."""
    n = 4
    src = torch.empty(n * piece, dtype=torch.uint8, pin_memory=True)
    hdst = torch.empty(n * piece, dtype=torch.uint8, pin_memory=True)
    dst = torch.empty(n * piece, dtype=torch.uint8, device="cuda:%d" % device)
    dsrc = torch.empty(n * piece, dtype=torch.uint8, device="cuda:%d" % device)
    s1, s2 = torch.cuda.Stream(device=device), torch.cuda.Stream(device=device)
    reps = max(1, (8 << 30) // (n * piece))

    def h2d(s):
        with torch.cuda.stream(s):
            for i in range(n):
                dst[i * piece:(i + 1) * piece].copy_(src[i * piece:(i + 1) * piece], non_blocking=True)

    def d2h(s):
        with torch.cuda.stream(s):
            for i in range(n):
                hdst[i * piece:(i + 1) * piece].copy_(dsrc[i * piece:(i + 1) * piece], non_blocking=True)

    def timed(dirs):
        e0 = torch.cuda.Event(enable_timing=True)
        e0.record(s1)
        s2.wait_event(e0)
        ends = []
        for s, f in dirs:
            for _ in range(reps):
                f(s)
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            ends.append(e)
        for e in ends:
            s1.wait_event(e)
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record(s1)
        e1.synchronize()
        return [e0.elapsed_time(e) * 1e-3 for e in ends], e0.elapsed_time(e1) * 1e-3

    h2d(s1)
    d2h(s2)                                               # warm-up
    torch.cuda.synchronize()
    nbytes = reps * n * piece
    # PASSES passes of each, interleaved; every figure is the best pass (the link's capability, so a
    # fraction of it stays <= 1 unless the workload beats the probe) with the median beside it: single
    # slow passes were seen (D2H once 30.6 vs 56.6 GB/s on a fresh box; a bidirectional pass 57.5 vs
    # 96.8 GB/s in round 5, which made a "fraction" of 1.40)
    hs, ds, bs = [], [], []
    for _ in range(PASSES):
        hs.append(timed([(s1, h2d)])[0][0])
        ds.append(timed([(s2, d2h)])[0][0])
        bs.append(timed([(s1, h2d), (s2, d2h)]))
    del src, hdst, dst, dsrc
    torch.cuda.empty_cache()
    (t_bh, t_bd), t_b = min(bs, key=lambda x: x[1])
    med = sorted(x[1] for x in bs)[len(bs) // 2]
    return {"h2d": nbytes / min(hs) / 1e9, "d2h": nbytes / min(ds) / 1e9, "bidir": 2 * nbytes / t_b / 1e9,
            "bidir_h2d": nbytes / t_bh / 1e9, "bidir_d2h": nbytes / t_bd / 1e9,
            "median": {"h2d": round(nbytes / sorted(hs)[len(hs) // 2] / 1e9, 2),
                       "d2h": round(nbytes / sorted(ds)[len(ds) // 2] / 1e9, 2),
                       "bidir": round(2 * nbytes / med / 1e9, 2)},
            "passes": PASSES,
            "bidir_passes_GB_s": [round(2 * nbytes / x[1] / 1e9, 1) for x in bs]}


def read_bench(ctx, dev, S, m, hasher, compressor):
    """Read side (DataConstructor, hdrf_reconstruct): m blocks of the same corpus reduced into a
    separate context that keeps recipes, then every block rebuilt into HBM from its recipe (index
    lookups + chunk gather from the container arena); checked byte for byte on the first block."""
    import numpy as np
    from hdrf_amd.lib import Context
    B = 8
    v = Context(device=int(ctx.cfg.device), hasher=hasher, compressor=compressor, max_block_bytes=S,
                max_batch_blocks=B, index_log2=24, arena_slots=512, keep_recipes=1)
    for b0 in range(0, m, B):
        k = min(B, m - b0)
        v.reduce_batch([dev + (b0 + i) * S for i in range(k)], [S] * k, [S + 4096] * k, list(range(b0, b0 + k)))
    recipes = [v.recipe(b) for b in range(m)]
    out = v.dev_alloc(S + 4096)
    v.reconstruct(recipes[0], out, S)                    # warm-up
    ok = bool(np.array_equal(v.d2h(out, S), ctx.d2h(dev, S)))
    t0 = time.perf_counter()
    for r in recipes:
        v.reconstruct(r, out, S)
    t = time.perf_counter() - t0
    v.dev_free(out)
    v.close()
    return {"GB_s": round(m * S / t / 1e9, 2), "blocks": m, "seconds": round(t, 4), "first_block_identical": ok,
            "path": "hdrf_reconstruct: recipe digests -> index lookup -> offsets scan -> arena gather, output in HBM, "
                    "one block per call (host round trip each)"}


def cpu_baseline(ctx, dev, S, m, gpu_store, hasher, compressor=1, gpu_res=None):
    """CPU oracle (C restatement of the reference) on the first m blocks of the same corpus, timed
    in BASELINE.md's two shapes plus one thread:
      reference  the reference's own concurrency, blocks serialised: per block 1 chunking thread,
                 3 threadedHasher threads over the chunk ranges, then the ordered index part and 3
                 concurrent threadedStorer threads (DN/DataDeduplicator.java:122-204, :578-641, :652-836)
      all_cores  every usable core (sched_getaffinity): chunk + hash of later blocks on N-1 worker
                 threads ahead of 1 ordered index/store thread
    All check per-block storeSize == the GPU's (bit-exact dedup ratio); the all-cores run also
    returns every block's chunk END offsets, digests and is_new, compared chunk by chunk with the
    GPU's (gpu_res); for the compression stage a fresh GPU context reducing the same m blocks
    must write byte-identical container files."""
    from oracle.oracle import Oracle
    blks = [ctx.d2h(dev + b * S, S) for b in range(m)]
    ids = list(range(m))
    usable = cpu_share()
    ora = Oracle(hasher=hasher, compressor=compressor)
    t0 = time.perf_counter()
    ss1 = [ora.reduce(blk, b)["store_size"] for b, blk in enumerate(blks)]
    t1 = time.perf_counter() - t0
    ref = Oracle(hasher=hasher, compressor=compressor)
    t0 = time.perf_counter()
    ssr = ref.reduce_ref_shape(blks, ids, 3)
    tr = time.perf_counter() - t0
    nthr = max(1, usable - 1)
    par = Oracle(hasher=hasher, compressor=compressor)
    t0 = time.perf_counter()
    full = par.reduce_many_full(blks, ids, nthr)
    tp = time.perf_counter() - t0
    ssp = [r["store_size"] for r in full]
    chunk_bad = {"offsets": 0, "digests": 0, "is_new": 0}
    n_chunks = 0
    for b, r in enumerate(full):
        g = gpu_res[b] if gpu_res is not None and b < len(gpu_res) else None
        n_chunks += len(r["offsets"])
        if g is None or len(g["offsets"]) != len(r["offsets"]):
            for k in chunk_bad:
                chunk_bad[k] += len(r["offsets"])
            continue
        chunk_bad["offsets"] += int((g["offsets"] != r["offsets"]).sum())
        chunk_bad["digests"] += int((g["digests"] != r["digests"]).any(axis=1).sum())
        chunk_bad["is_new"] += int((g["is_new"] != r["is_new"]).sum())

    def mism(ss):
        return int(sum(int(ss[b] != gpu_store[b]) for b in range(m)))

    sample = "first %d of the same blocks (%.1f GiB), oracle/hdrf_oracle.c%s" % (
        m, m * S / 2**30, " with lz4 r123 containers" if compressor == 2 else "")
    out = {"value": round(m * S / tp / 1e9, 4), "unit": "GB/s", "cores": nthr + 1, "kind": "port",
           "sample": sample + ", all usable cores: %d chunk+hash worker threads + 1 ordered index thread with 3 "
                              "concurrent storer threads per block, %.1f s" % (nthr, tp),
           "store_size_mismatches": mism(ssp),
           "chunk_check": {"blocks": m, "chunks": n_chunks, "mismatches": chunk_bad,
                           "what": "per chunk: END offset, digest, is_new (GPU from a fresh index over the same "
                                   "batches vs the oracle in block order)"},
           "cpu_model": _cpu_model(), "nproc": os.cpu_count(),
           "usable_cores": usable,
           "reference_shape": {"value": round(m * S / tr / 1e9, 4), "unit": "GB/s", "cores": 4,
                               "threads": "per block 1 chunking + 3 hasher threads, then the ordered part with 3 "
                                          "concurrent storer threads (each closing%s its own containers); blocks "
                                          "serialised" % (" and LZ4-compressing" if compressor == 2 else ""),
                               "seconds": round(tr, 2),
                               "store_size_mismatches": mism(ssr)},
           "single_thread": {"value": round(m * S / t1 / 1e9, 4), "unit": "GB/s", "cores": 1,
                             "seconds": round(t1, 2), "store_size_mismatches": mism(ss1)}}
    if compressor == 2:
        out["container_file_mismatches"], out["containers_checked"] = _check_containers(ctx, dev, S, m, ora, hasher)
    return out


def cpu_share():
    """Host cores this process may use: the affinity mask, capped by a cgroup CPU quota (a GPU box
    shows the whole machine's CPUs but grants each GPU a share of them)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def corpus_check(ctx, dev, S, nb, B, gpu_store, hasher, compressor, host=None):
    """Every block's storeSize from the timed steps (DN/DataDeduplicator.java:355: the bytes a block
    adds to the containers) against the oracle over the whole corpus in block order, so the line's
    dedup ratio is checked bit for bit, not only on a sample.  The oracle runs in store-size mode
    (container lengths, no container or recipe bytes in host memory) on the threaded baseline's
    shape, fed one pinned batch at a time."""
    import numpy as np
    from oracle.oracle import Oracle
    ora = Oracle(hasher=hasher, compressor=compressor, store_only=True)
    nthr = max(1, cpu_share() - 1)
    buf = ctx.host_alloc(B * S) if host is None else None
    ss = []
    t0 = time.perf_counter()
    for b0 in range(0, nb, B):
        k = min(B, nb - b0)
        if host is None:
            ctx.L.hdrf_memcpy_d2h(ctx._h, buf.ctypes.data, dev + b0 * S, k * S)
            src = buf
        else:
            src = host[b0 * S:(b0 + k) * S]
        ss.extend(int(x) for x in ora.reduce_many([src[i * S:(i + 1) * S] for i in range(k)],
                                                   list(range(b0, b0 + k)), nthr))
    t = time.perf_counter() - t0
    if buf is not None:
        ctx.host_free(buf)
    ss = np.array(ss, np.int64)
    stored = int(ss.sum())
    gpu = np.asarray(gpu_store[:nb], np.int64)
    return {"blocks": nb, "store_size_mismatches": int((ss != gpu).sum()),
            "stored_bytes_oracle": stored, "stored_bytes_gpu": int(gpu.sum()),
            "dedup_ratio_oracle": round(nb * S / max(stored, 1), 6),
            "dedup_ratio_gpu": round(nb * S / max(int(gpu.sum()), 1), 6),
            "seconds": round(t, 1), "threads": nthr + 1,
            "what": "every block's storeSize of the last timed step vs oracle/hdrf_oracle.c in store-size mode "
                    "(the whole corpus in block order from a fresh index; untimed)"}


def _check_containers(ctx, dev, S, m, ora, hasher):
    from hdrf_amd.lib import Context
    v = Context(device=int(ctx.cfg.device), hasher=hasher, compressor=2, max_block_bytes=S, max_batch_blocks=8,
                index_log2=24, arena_slots=256, keep_recipes=0)
    for b0 in range(0, m, 8):
        k = min(8, m - b0)
        v.reduce_batch([dev + (b0 + i) * S for i in range(k)], [S] * k, [S + 4096] * k, list(range(b0, b0 + k)))
    alloc = ora.allocator()
    bad = checked = 0
    for t in range(3):
        last = int.from_bytes(alloc[3 * t:3 * t + 3], "big")
        for cid in range(t << 22, last + 1):
            od, oc = ora.container(cid)
            if od is None:
                continue
            gd, gc = v.container(cid)
            checked += 1
            bad += int(gd != od or gc != oc)
    v.close()
    return bad, checked


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
