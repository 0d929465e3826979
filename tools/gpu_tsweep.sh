#!/bin/bash
# GPU-box: all gpu tests, then a knob sweep on hg19 + hg19r: tools/gpu_tsweep.sh TAG VAR v1 v2 ...
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
bash tools/gpu_sweep.sh $TAG "$@"
