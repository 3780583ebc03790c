# Round 5, call 8: GPU suite on the window-pair verification, LZ4 tests on the streaming-store build,
# config-4 A/B of the three, phase profile
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_g.log 2>&1 || { tail -30 gpurun_out/r05_tests_g.log; exit 1; }
tail -1 gpurun_out/r05_tests_g.log
HDRF_LIB_PATH=hdrf_amd/_build_ntout/libhdrf.so timeout -k 10 300 python -u -m pytest tests/test_lz4.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_g_nt.log 2>&1 || { tail -30 gpurun_out/r05_tests_g_nt.log; exit 1; }
tail -1 gpurun_out/r05_tests_g_nt.log
TAG=r05_lz4c bash scripts/abrun.sh scripts/ab_r05_lz4c.txt || exit 1
HDRF_LIB_PATH=hdrf_amd/_build_prof/libhdrf.so HDRF_LZ4_PHASES=1 timeout -k 10 300 python -u bench.py --workload config4 \
  --steps 1 --warmup 1 --no-cpu --no-alone --no-sub > gpurun_out/r05_lzp_c.json.log 2>&1 || { tail -20 gpurun_out/r05_lzp_c.json.log; exit 1; }
tail -1 gpurun_out/r05_lzp_c.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d['roofline']['lz4'].get('phases_in_pipeline') or {}
print('c', d['value'], json.dumps(p))"
