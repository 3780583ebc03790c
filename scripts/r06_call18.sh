#!/bin/bash
# Round 6, call 18: counted traffic and VALU instructions of the fused front (HDRF_FUSED=1) on config 2
# (FETCH_SIZE, WRITE_SIZE, SQ_INSTS_VALU + SQ_WAVES passes, one counter group per rocprofv3 run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
HDRF_FUSED=1 EXTRA_GROUPS="SQ_INSTS_VALU SQ_WAVES" ARGS="--steps 1 --warmup 0 --no-cpu --no-alone --no-sub --no-corpus-check" \
  TAG=r06_fz bash scripts/r02_traffic.sh > gpurun_out/r06_fz_traffic.log 2>&1 || { tail -20 gpurun_out/r06_fz_traffic.log; exit 1; }
python3 - <<'PY'
import json
d = json.load(open('gpurun_out/r06_fz_traffic.json'))
tot = 0
for k, v in sorted(d.items(), key=lambda kv: -(kv[1].get('hbm_bytes_per_launch', 0) if isinstance(kv[1], dict) else 0)):
    if isinstance(v, dict) and 'hbm_bytes_per_launch' in v:
        print('%-34s %8.3f GB  valu %s' % (k, v['hbm_bytes_per_launch'] / 1e9, v.get('sq_insts_valu')))
PY
