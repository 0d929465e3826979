#!/bin/bash
# C2 (hg19) knob re-check on the final kernels: run-ahead depth and the report-batch threshold
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 500 python -u tools/knob_sweep.py --genome hg19 --reads 10000000 --steps 2 --var multi \
  "GWA_RUNAHEAD=4" "GWA_RUNAHEAD=3" "GWA_RUNAHEAD=6" "GWA_WAITQ16=12" "GWA_WAITQ16=16" "GWA_RUNAHEAD=4" > gpurun_out/knobs_c2.log 2>&1
