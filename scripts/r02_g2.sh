# 2-rank rehearsal of the node-global bench on one GPU (gloo): allocator scan, then the chain
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for mode in scan chain; do
  if [ $mode = chain ]; then export HDRF_NODE_CHAIN=1; fi
  HDRF_BENCH_SAME_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29655 bench.py --gpus 2 --steps 2 --warmup 1 --blocks 64 --no-cpu > gpurun_out/g2_$mode.log 2>&1 || { tail -30 gpurun_out/g2_$mode.log; exit 1; }
  tail -1 gpurun_out/g2_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', d['value'], d['ms_per_step'], d['node_back_ms_per_batch'])"
done
