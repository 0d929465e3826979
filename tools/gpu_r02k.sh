#!/bin/bash
# GPU-box: all gpu tests, then a C5 (paired-end) bench line.
set -o pipefail
TAG=${1:-r02k}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 900 python -u bench.py --workload c5 "$@" > gpurun_out/${TAG}_bench_c5.json 2> gpurun_out/${TAG}_bench_c5.err || { tail -30 gpurun_out/${TAG}_bench_c5.err; exit 1; }
cat gpurun_out/${TAG}_bench_c5.json
