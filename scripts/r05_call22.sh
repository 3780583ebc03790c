# Round 5, call 22: the LZ4 parse phases inside the config-4 pipeline at HEAD (profiling build)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
HDRF_LIB_PATH=hdrf_amd/_build_prof/libhdrf.so HDRF_LZ4_PHASES=1 timeout -k 10 300 python -u bench.py --workload config4 \
  --steps 1 --warmup 1 --no-cpu --no-alone --no-sub > gpurun_out/r05_lzp_d.json.log 2>&1 || { tail -20 gpurun_out/r05_lzp_d.json.log; exit 1; }
tail -1 gpurun_out/r05_lzp_d.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d['roofline']['lz4'].get('phases_in_pipeline') or {}
print('d', d['value'], json.dumps(p))"
