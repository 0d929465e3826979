#!/bin/bash
# round-4 final measurement, part B: the secondary bench lines and a C4 -m bsf kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
bash tools/lines.sh r04b || exit $?
PASS=trace bash tools/profile.sh r04b_c4 --workload c4 --steps 3 --warmup 1
