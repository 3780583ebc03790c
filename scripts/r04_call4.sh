#!/bin/bash
# Round 4: LZ4 variant A/B on config 4 (default = v1: 2-bit table tags; v3 = + DPP collision check;
# v4 = + non-returning table updates; fb4 / fb16 = first search batch of 4 / 16 attempts), alternated.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
P=hdrf_amd
NO_TESTS=1 V=d VARIANTS="X=new HDRF_LIB_PATH=$P/_build_v3/libhdrf.so HDRF_LIB_PATH=$P/_build_v4/libhdrf.so HDRF_LIB_PATH=$P/_build_fb4/libhdrf.so HDRF_LIB_PATH=$P/_build_fb16/libhdrf.so X=new HDRF_LIB_PATH=$P/_build_v3/libhdrf.so HDRF_LIB_PATH=$P/_build_v4/libhdrf.so HDRF_LIB_PATH=$P/_build_fb4/libhdrf.so HDRF_LIB_PATH=$P/_build_fb16/libhdrf.so" bash scripts/r04_lz4ab.sh
