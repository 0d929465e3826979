#!/bin/bash
# GPU-box: the secondary bench lines (hg19r C2, C4 bsf / sf, C5 paired-end) into gpurun_out/lines_TAG/
set -o pipefail
TAG=$1
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
D=gpurun_out/lines_$TAG
mkdir -p $D
run() { name=$1; shift; timeout -k 10 500 python3 -u bench.py "$@" > $D/$name.json 2> $D/$name.err || { tail -20 $D/$name.err; exit 1; }; echo "== $name"; cut -c1-400 $D/$name.json; }
run c2_hg19r --genome hg19r --no-pipeline
run c4_bsf --workload c4 --no-pipeline
run c4_sf --workload c4 --strategy sf --no-pipeline
run c5 --workload c5
