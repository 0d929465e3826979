#!/bin/bash
# GPU-box: sweep one env knob on hg19 and hg19r C2 (tools/knob_sweep.py): gpu_knob.sh TAG VAR v1 v2 ...
set -o pipefail
TAG=$1; VAR=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
for g in hg19 hg19r; do
timeout -k 10 400 python -u tools/knob_sweep.py --genome $g --steps 2 --var $VAR "$@" > gpurun_out/${TAG}_$g.log 2>&1 || { tail -20 gpurun_out/${TAG}_$g.log; exit 1; }
cat gpurun_out/${TAG}_$g.log
done
