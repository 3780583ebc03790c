# Round 5, call 24: GPU suite on HEAD (codec options); LZ4 tests on the scheduling-strategy builds; config-4 A/B
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_s.log 2>&1 || { tail -30 gpurun_out/r05_tests_s.log; exit 1; }
tail -1 gpurun_out/r05_tests_s.log
for b in ilp mc iilp; do
  HDRF_LIB_PATH=hdrf_amd/_build_$b/libhdrf.so timeout -k 10 300 python -u -m pytest tests/test_lz4.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_s_$b.log 2>&1 || { tail -30 gpurun_out/r05_tests_s_$b.log; exit 1; }
  echo "$b $(tail -1 gpurun_out/r05_tests_s_$b.log)"
done
TAG=r05_sched bash scripts/abrun.sh scripts/ab_r05_sched.txt || exit 1
