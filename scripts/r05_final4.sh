#!/bin/bash
# Round 5 closing run d (sha_carry the default): GPU suite, smoke, the default bench line as the driver runs it,
# the config-4 line with its CPU leg, config 5 whole blocks (c1, c2), then rocprofv3 kernel-trace summaries of the config-2 and config-4 pipelines
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
V=${V:-final_d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r05_tests_$V.log 2>&1 || { tail -40 gpurun_out/r05_tests_$V.log; exit 1; }
tail -1 gpurun_out/r05_tests_$V.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_smoke_$V.log 2>&1 || { tail -20 gpurun_out/r05_smoke_$V.log; exit 1; }
tail -1 gpurun_out/r05_smoke_$V.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 2 > gpurun_out/r05_bench_$V.json.log 2>&1 || { tail -20 gpurun_out/r05_bench_$V.json.log; exit 1; }
tail -1 gpurun_out/r05_bench_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']
print('bench', d['value'], 'period', r.get('batch_period_ms'), 'frac', r.get('frac'), ' '.join('%s=%s' % (k, v.get('value')) for k, v in (d.get('configs') or {}).items()))"
timeout -k 10 600 python -u bench.py --workload config4 > gpurun_out/r05_c4_$V.json.log 2>&1 || { tail -20 gpurun_out/r05_c4_$V.json.log; exit 1; }
tail -1 gpurun_out/r05_c4_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d['roofline']; c=d['cpu_baseline']
print('c4', d['value'], 'period', r.get('batch_period_ms'), 'containers', c.get('container_file_mismatches'), '/', c.get('containers_checked'))"
for cmp in 1 2; do
  timeout -k 10 600 python -u bench.py --workload config5 --steps 3 --compressor $cmp > gpurun_out/r05_c5_whole_c${cmp}_$V.json.log 2>&1 || { tail -20 gpurun_out/r05_c5_whole_c${cmp}_$V.json.log; exit 1; }
  tail -1 gpurun_out/r05_c5_whole_c${cmp}_$V.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); p=d.get('pcie') or {}
print('c5 whole c$cmp', d['value'], 'v/bidir', p.get('value_over_bidirectional_raw'))"
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_prof_c2d -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-sub --no-cpu --no-alone > $R/gpurun_out/r05_prof_c2d.log 2>&1) || { echo "c2 trace failed"; tail -20 gpurun_out/r05_prof_c2d.log; exit 1; }
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05_prof_c4d -o run -- python3 $R/bench.py --workload config4 --steps 2 --warmup 1 --no-sub --no-cpu --no-alone > $R/gpurun_out/r05_prof_c4d.log 2>&1) || { echo "c4 trace failed"; tail -20 gpurun_out/r05_prof_c4d.log; exit 1; }
echo traces ok
