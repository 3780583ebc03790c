#!/bin/bash
# A/B of bench variants: each line is "ENV ARGS"; prints value + key stage times per variant.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
i=0
while IFS= read -r v; do
  [ -z "$v" ] && continue
  i=$((i+1))
  env $(echo "$v" | cut -d'|' -f1) timeout -k 10 300 python3 -u bench.py --no-cpu $(echo "$v" | cut -d'|' -f2) > gpurun_out/ab$i.log 2>&1 || { echo "variant $i failed: $v"; tail -5 gpurun_out/ab$i.log; exit 1; }
  python3 - gpurun_out/ab$i.log "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = d["stages"]
short = {k.split("(")[0]: v["avg_launch_ms"] for k, v in st.items()}
print(sys.argv[2], "=>", d["value"], "GB/s", {k: v for k, v in short.items() if v > 0.05})
if "alone" in d["roofline"]:
    print("   alone:", {k.split("(")[0]: v.get("avg_launch_ms", v.get("avg_batch_ms")) for k, v in d["roofline"]["alone"].items()})
PY
done < ${VARIANTS:-/dev/stdin}
