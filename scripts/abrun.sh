#!/bin/bash
# A/B runs of bench.py: one variant per line of the file $1 ("ENV=.. ENV2=..|bench args"), in file
# order (alternate the variants in the file); prints value, the per-stream chains and the period.
# Logs: gpurun_out/${TAG:-ab}_<n>.json.log
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
TAG=${TAG:-ab}
i=0
while IFS= read -r line; do
  [ -z "$line" ] && continue
  case "$line" in \#*) continue;; esac
  i=$((i+1))
  envs=${line%%|*}; args=${line#*|}
  env $envs timeout -k 10 400 python -u bench.py $args > gpurun_out/${TAG}_$i.json.log 2>&1 || { echo "variant $i ($line) failed"; tail -20 gpurun_out/${TAG}_$i.json.log; exit 1; }
  tail -1 gpurun_out/${TAG}_$i.json.log | python3 -c "
import json,sys
d=json.load(sys.stdin); r=d.get('roofline') or {}
ch=r.get('chains_ms_per_batch') or {}
print('%2d %-58s %9.2f  period %.3f  %s' % ($i, '''$line'''[:58], d['value'], r.get('batch_period_ms') or 0,
      ' '.join('%s=%.2f' % (k.split(':')[0], v) for k, v in ch.items())), flush=True)"
done < "$1"
