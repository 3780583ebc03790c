# LZ4 parse phase profile (profiling build under hdrf_amd/_build_prof)
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/lz4_prof.py > gpurun_out/lzp.log 2>&1; rc=$?
cat gpurun_out/lzp.log | grep -v "^W2026\|^E2026"; exit $rc
