# Round 5, call 5: GPU suite on the LZ4 chain change, config-4 A/B against the previous lz4.hip,
# and the per-phase shader-clock profile of the LZ4 parse inside the config-4 pipeline (both builds)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_d.log 2>&1 || { tail -30 gpurun_out/r05_tests_d.log; exit 1; }
tail -1 gpurun_out/r05_tests_d.log
TAG=r05_lz4ab bash scripts/abrun.sh scripts/ab_r05_lz4.txt || exit 1
for v in prof_prev prof; do
  HDRF_LIB_PATH=hdrf_amd/_build_$v/libhdrf.so HDRF_LZ4_PHASES=1 timeout -k 10 300 python -u bench.py --workload config4 \
    --steps 1 --warmup 1 --no-cpu --no-alone --no-sub > gpurun_out/r05_lzp_$v.json.log 2>&1 || { tail -20 gpurun_out/r05_lzp_$v.json.log; exit 1; }
  tail -1 gpurun_out/r05_lzp_$v.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d['roofline']['lz4'].get('phases_in_pipeline') or {}
print('$v', d['value'], json.dumps(p))"
done
