#!/bin/bash
# C4 -m bsf: lanes per tier with the round-4 hit lists (knob_sweep, SAM compared)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 600 python -u tools/knob_sweep.py --genome hg19 --c4 --k 5 --reads 1000000 --steps 2 --var multi \
  "GWA_TIER_LANES=262144,131072,65536,1024" "GWA_TIER_LANES=262144,65536,65536,1024" "GWA_TIER_LANES=262144,262144,65536,1024" \
  "GWA_TIER_LANES=131072,131072,65536,1024" "GWA_TIER_LANES=262144,131072,65536,1024" > gpurun_out/lanes_c4.log 2>&1
