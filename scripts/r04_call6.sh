#!/bin/bash
# Round 4: LZ4 variant A/B (config 4), then the config-2 knob A/B.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/r04_call4.sh || exit 1
bash scripts/r04_knobs.sh
