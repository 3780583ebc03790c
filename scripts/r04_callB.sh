#!/bin/bash
# Round 4: LZ4 speculative window pair — parity (LZ4 / compressor-2 / stream tests), then config-4 A/B
# against the committed build (hdrf_amd/_build_v4c), alternated.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
P=hdrf_amd
V=s VARIANTS="X=new HDRF_LIB_PATH=$P/_build_v4c/libhdrf.so X=new HDRF_LIB_PATH=$P/_build_v4c/libhdrf.so X=new HDRF_LIB_PATH=$P/_build_v4c/libhdrf.so" bash scripts/r04_lz4ab.sh
