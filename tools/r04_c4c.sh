#!/bin/bash
# C4 -m bsf: tier-1 capacities (knob_sweep, SAM compared; GWA_VERBOSE prints each tier's overflow bits)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
GWA_VERBOSE=1 timeout -k 10 900 python -u tools/knob_sweep.py --genome hg19 --c4 --k 5 --reads 1000000 --steps 1 --var multi \
  "GWA_TIER_JUMP=1" "GWA_TIER_ARENA=256,2048,4096,65536" "GWA_TIER_ARENA=256,4096,4096,65536" \
  "GWA_TIER_HITS=128,512,256,4096;GWA_TIER_CIGAR=2048,8192,4096,65536" \
  "GWA_TIER_ARENA=512,1024,4096,65536" "GWA_TIER_LANES=262144,131072,65536,1024;GWA_SPARSE_LANES=65536" \
  > gpurun_out/sweep_c4c.log 2>&1
