#!/bin/bash
# GPU-box: quick-scan / search time at k-mer table sizes GWA_KMER_K (hg19-size C2 and hg19r)
set -o pipefail
TAG=${1:-kmer}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
for K in "$@"; do
for g in hg19 hg19r; do
GWA_KMER_K=$K timeout -k 10 300 python -u tools/knob_sweep.py --genome $g --steps 2 --var X - > gpurun_out/${TAG}_${g}_$K.log 2>&1 || { tail -20 gpurun_out/${TAG}_${g}_$K.log; exit 1; }
echo "K=$K $g $(grep X= gpurun_out/${TAG}_${g}_$K.log)"
done
done
