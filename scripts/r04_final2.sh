#!/bin/bash
# Round 4 closing run, part 2: config-4 traffic at HEAD and its bench line, the config-5 lines
# (whole blocks and 64 KiB packets with mirroring, compressor 1 and 2) and the two-rank rehearsal.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out profiles
V=${V:-f}
TAG=r04_c4$V WORKLOAD=config4 ARGS="--workload config4 --steps 1 --warmup 0 --no-cpu --no-alone" bash scripts/r02_traffic.sh > gpurun_out/r04_c4traffic_$V.txt 2>&1 || { tail -20 gpurun_out/r04_c4traffic_$V.txt; exit 1; }
cp gpurun_out/r04_c4${V}_traffic.json profiles/r04_c4${V}_traffic.json
timeout -k 10 600 python -u bench.py --workload config4 > gpurun_out/r04_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_c4_$V.json.log | cut -c1-200
timeout -k 10 400 python -u bench.py --workload config5 --steps 3 > gpurun_out/r04_c5_whole_c1_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_c5_whole_c1_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_c5_whole_c1_$V.json.log | cut -c1-200
timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --compressor 2 > gpurun_out/r04_c5_whole_c2_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_c5_whole_c2_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_c5_whole_c2_$V.json.log | cut -c1-200
timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 1 > gpurun_out/r04_c5_pk64_c1_ring_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_c5_pk64_c1_ring_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_c5_pk64_c1_ring_$V.json.log | cut -c1-200
timeout -k 10 400 python -u bench.py --workload config5 --steps 3 --packet-driver cpp --packet-kib 64 --mirror ring --compressor 2 > gpurun_out/r04_c5_pk64_c2_ring_$V.json.log 2>&1 || { tail -20 gpurun_out/r04_c5_pk64_c2_ring_$V.json.log; exit 1; }
tail -1 gpurun_out/r04_c5_pk64_c2_ring_$V.json.log | cut -c1-200
# the multi-rank path: two ranks on this one GPU over gloo (a rehearsal of bench.py --gpus N, not a
# measurement: both ranks share the device)
HDRF_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --steps 2 --warmup 1 --blocks 64 --no-cpu > gpurun_out/r04_g2_$V.log 2>&1 || { tail -30 gpurun_out/r04_g2_$V.log; exit 1; }
tail -1 gpurun_out/r04_g2_$V.log | cut -c1-300
