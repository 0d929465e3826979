#!/bin/bash
# C4 -m bsf: the k >= 4 report-batch threshold on the round-4 tiers (knob_sweep, SAM compared)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 600 python -u tools/knob_sweep.py --genome hg19 --c4 --k 5 --reads 1000000 --steps 2 --var GWA_WAITQ16 8 6 10 8 6 > gpurun_out/wq_c4b.log 2>&1
