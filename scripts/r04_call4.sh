#!/bin/bash
# Round 4: LZ4 tag variants A/B (v1 default = tags; v3 = + DPP collision check; v4 = + non-returning
# table updates), then the config-5 lines and config 4 on the default build.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
P=hdrf_amd
NO_TESTS=1 V=d VARIANTS="X=new HDRF_LIB_PATH=$P/_build_v3/libhdrf.so HDRF_LIB_PATH=$P/_build_v4/libhdrf.so X=new HDRF_LIB_PATH=$P/_build_v3/libhdrf.so HDRF_LIB_PATH=$P/_build_v4/libhdrf.so" bash scripts/r04_lz4ab.sh || exit 1
V=a bash scripts/r04_c5.sh
