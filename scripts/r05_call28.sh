# Round 5, call 28: sha_carry as the default: GPU suite, config-4 A/B, config-2 traffic (FETCH / WRITE passes)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05_tests_u.log 2>&1 || { tail -30 gpurun_out/r05_tests_u.log; exit 1; }
tail -1 gpurun_out/r05_tests_u.log
TAG=r05_carry4 bash scripts/abrun.sh scripts/ab_r05_carry4.txt || exit 1
TAG=r05_c2b ARGS="--steps 1 --warmup 0 --no-cpu --no-alone --no-sub" bash scripts/r02_traffic.sh || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r05_c2b_traffic.json'))
print({k: round(v['hbm_bytes_per_launch']/1e9, 3) for k, v in d.items() if not k.startswith('_') and v['hbm_bytes_per_launch'] > 1e8})"
