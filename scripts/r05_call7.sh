# Round 5, call 7: GPU suite on the search / extension restructure, config-4 A/B, phase profile
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_f.log 2>&1 || { tail -30 gpurun_out/r05_tests_f.log; exit 1; }
tail -1 gpurun_out/r05_tests_f.log
TAG=r05_lz4b bash scripts/abrun.sh scripts/ab_r05_lz4b.txt || exit 1
HDRF_LIB_PATH=hdrf_amd/_build_prof/libhdrf.so HDRF_LZ4_PHASES=1 timeout -k 10 300 python -u bench.py --workload config4 \
  --steps 1 --warmup 1 --no-cpu --no-alone --no-sub > gpurun_out/r05_lzp_b.json.log 2>&1 || { tail -20 gpurun_out/r05_lzp_b.json.log; exit 1; }
tail -1 gpurun_out/r05_lzp_b.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d['roofline']['lz4'].get('phases_in_pipeline') or {}
print('b', d['value'], json.dumps(p))"
TAG=r05_batch bash scripts/abrun.sh scripts/ab_r05_batch.txt || exit 1
