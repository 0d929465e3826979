#!/bin/bash
# C4 -m bsf: verification memo and first-tier hit-list capacities (knob_sweep, SAM compared)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 900 python -u tools/knob_sweep.py --genome hg19 --c4 --k 5 --reads 1000000 --steps 2 --var multi \
  "GWA_VERIFY_MEMO=0" "GWA_VERIFY_MEMO=1" \
  "GWA_TIER_HITS=128,256,256,4096;GWA_TIER_CIGAR=2048,4096,4096,65536" \
  "GWA_TIER_HITS=128,256,256,4096;GWA_TIER_CIGAR=2048,4096,4096,65536;GWA_TIER_ARENA=512,1024,4096,65536" \
  "GWA_TIER_HITS=256,256,256,4096;GWA_TIER_CIGAR=4096,4096,4096,65536;GWA_TIER_ARENA=512,2048,4096,65536" \
  "GWA_TIER_HITS=128,256,256,4096;GWA_TIER_CIGAR=2048,4096,4096,65536;GWA_VERIFY_MEMO=0" \
  > gpurun_out/sweep_c4.log 2>&1
