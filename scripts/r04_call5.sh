#!/bin/bash
# Round 4: the config-5 lines (mirrored packet driver c1/c2, batched submits, whole blocks c1/c2,
# link probes) and config 4, then the SHA line ring (parity + config-2 A/B).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
V=a bash scripts/r04_c5.sh || exit 1
V=a bash scripts/r04_sha_ring.sh
