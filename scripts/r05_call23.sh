# Round 5, call 23: the structurizer option on the stream codecs and the read side (gzip, inflate, snappy, lzo,
# read): GPU suite on that build, then codec timings A/B (HEAD vs _build_codec, alternating)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
HDRF_LIB_PATH=hdrf_amd/_build_codec/libhdrf.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_r.log 2>&1 || { tail -30 gpurun_out/r05_tests_r.log; exit 1; }
tail -1 gpurun_out/r05_tests_r.log
for v in head codec head codec; do
  if [ $v = codec ]; then L=hdrf_amd/_build_codec/libhdrf.so; else L=hdrf_amd/_build/libhdrf.so; fi
  echo "== $v"
  HDRF_LIB_PATH=$L timeout -k 10 300 python -u scripts/codec_ab.py 32 2>&1 | grep -v "^W2026\|^E2026" || exit 1
done
