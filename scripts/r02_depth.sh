# depth / stream-priority A/B of the config-2 pipeline
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for p in 1 2; do for d in 2 3; do
  HDRF_PRIO=$p timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 1 --depth $d > gpurun_out/depth${d}_p$p.log 2>&1 || { tail -20 gpurun_out/depth${d}_p$p.log; exit 1; }
  tail -1 gpurun_out/depth${d}_p$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('prio $p depth $d', d['value'], d['ms_per_step'], r['chains_ms_per_batch'], r['batch_period_ms'])"
done; done
