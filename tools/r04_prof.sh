#!/bin/bash
# Round-4 profiles: default bench (trace + 4 PMC passes), C4 -m bsf trace + FETCH/WRITE passes, profiling-build regions
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
bash tools/profile.sh r04 --steps 5 --warmup 2 || exit $?
PASS=trace bash tools/profile.sh r04_c4 --workload c4 --steps 3 --warmup 1 || exit $?
bash tools/gpu_prof.sh
