#!/bin/bash
# footprint experiment: C2 (hg19) and C4 -m bsf search time against padding added to every lane's slice
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 500 python -u tools/knob_sweep.py --genome hg19 --reads 10000000 --steps 2 --var GWA_SLICE_PAD 0 32768 131072 0 > gpurun_out/pad_c2.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/knob_sweep.py --genome hg19 --c4 --k 5 --reads 1000000 --steps 1 --var GWA_SLICE_PAD 0 131072 0 > gpurun_out/pad_c4.log 2>&1
