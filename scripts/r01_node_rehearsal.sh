#!/bin/bash
# One-GPU rehearsal of the multi-rank bench path (2 ranks on cuda:0 over gloo) + the N=1 bench.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
HDRF_BENCH_SAME_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29701 bench.py --gpus 2 --blocks 16 --batch 8 --block-mib 32 --steps 2 --warmup 1 --no-cpu --index-log2 23 > gpurun_out/rehearsal2.log 2>&1 || { echo "rehearsal failed"; tail -30 gpurun_out/rehearsal2.log; exit 1; }
grep '^{' gpurun_out/rehearsal2.log | tail -1 | cut -c1-900
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/bench1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench1.log; exit 1; }
tail -1 gpurun_out/bench1.log | cut -c1-600
