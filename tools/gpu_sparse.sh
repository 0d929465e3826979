#!/bin/bash
# GPU-box: gpu tests, then one-read-per-wavefront deep tiers on / off (GWA_SPARSE_LANES=1 turns it off)
set -o pipefail
TAG=${1:-sp}
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u tools/knob_sweep.py --genome hg19r --steps 2 --var GWA_SPARSE_LANES - 16384 1 > gpurun_out/${TAG}_hg19r.log 2>&1 || { tail -20 gpurun_out/${TAG}_hg19r.log; exit 1; }
grep GWA_ gpurun_out/${TAG}_hg19r.log
timeout -k 10 400 python -u tools/knob_sweep.py --genome hg19 --c4 --k 5 --reads 1000000 --steps 1 --var GWA_SPARSE_LANES - 16384 1 > gpurun_out/${TAG}_c4.log 2>&1 || { tail -20 gpurun_out/${TAG}_c4.log; exit 1; }
grep GWA_ gpurun_out/${TAG}_c4.log
