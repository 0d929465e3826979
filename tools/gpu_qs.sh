#!/bin/bash
# GPU-box: gpu parity tests, then quick-scan / search times on hg19 and hg19r (knob_sweep, no knob)
set -o pipefail
TAG=${1:-qs}
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for g in hg19 hg19r; do
timeout -k 10 300 python -u tools/knob_sweep.py --genome $g --steps 2 --var X - > gpurun_out/${TAG}_$g.log 2>&1 || { tail -20 gpurun_out/${TAG}_$g.log; exit 1; }
echo "$g $(grep X= gpurun_out/${TAG}_$g.log)"
done
