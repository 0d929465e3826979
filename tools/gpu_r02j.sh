#!/bin/bash
# GPU-box: all gpu tests, then the hg19r bench line (no CPU legs).
set -o pipefail
TAG=${1:-r02j}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 900 python -u bench.py --genome hg19r --no-cpu "$@" > gpurun_out/${TAG}_bench_hg19r.json 2> gpurun_out/${TAG}_bench_hg19r.err || { tail -30 gpurun_out/${TAG}_bench_hg19r.err; exit 1; }
cat gpurun_out/${TAG}_bench_hg19r.json
