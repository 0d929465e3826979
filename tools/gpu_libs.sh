#!/bin/bash
# GPU-box: the same C2 batch under several builds of the library: tools/gpu_libs.sh TAG GENOME lib1.so lib2.so ...
set -o pipefail
TAG=$1; G=$2; shift 2
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
for l in "$@"; do
GWA_LIB=$l timeout -k 10 400 python -u tools/knob_sweep.py --genome $G --steps 2 $KS_ARGS --var X - > gpurun_out/${TAG}_$l.log 2>&1 || { tail -20 gpurun_out/${TAG}_$l.log; exit 1; }
echo "== $l"; grep "X=" gpurun_out/${TAG}_$l.log
done
