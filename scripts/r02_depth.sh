# depth / hardware-queue A/B of the config-2 pipeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for q in 4 8; do for d in 2 3; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 1 --depth $d > gpurun_out/depth${d}_q$q.log 2>&1 || { tail -20 gpurun_out/depth${d}_q$q.log; exit 1; }
  tail -1 gpurun_out/depth${d}_q$q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('q $q depth $d', d['value'], d['ms_per_step'], r['chains_ms_per_batch'], r['batch_period_ms'])"
done; done
