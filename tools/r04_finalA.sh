#!/bin/bash
# round-4 final measurement, part A: smoke(), then the default bench under rocprofv3 (trace + four PMC passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out/final
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit $?
bash tools/profile.sh r04b
