#!/bin/bash
# GPU-box: tier lane-budget sweep (GWA_TIER_LANES) on C4 -m bsf and C2 hg19r.
set -o pipefail
TAG=${1:-tiers}
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/knob_sweep.py --genome hg19 --c4 --k 5 --reads 1000000 --steps 1 --var GWA_TIER_HITS - 0,256,0,0 0,256,1024,0 0,1024,4096,0 > gpurun_out/${TAG}_c4.log 2>&1 || { tail -20 gpurun_out/${TAG}_c4.log; exit 1; }
cat gpurun_out/${TAG}_c4.log
