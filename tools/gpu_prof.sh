#!/bin/bash
# GPU-box: search-kernel region profile (profiling build) on hg19 and hg19r, C2 reads.
set -o pipefail
TAG=${1:-prof}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
for g in hg19 hg19r; do
GWA_LIB=libgwa_prof.so timeout -k 10 400 python -u tools/knob_sweep.py --genome $g --steps 1 --var X - > gpurun_out/${TAG}_$g.log 2>&1 || { tail -20 gpurun_out/${TAG}_$g.log; exit 1; }
cat gpurun_out/${TAG}_$g.log
done
