#!/bin/bash
# GPU-box check: gpu tests, default bench without the CPU legs, end-to-end CLI timing.
set -o pipefail
TAG=${1:-r02c}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python -u bench.py --no-cpu "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 600 python -u tools/e2e_cli.py --reads 6000000 --saved-index > gpurun_out/${TAG}_e2e.log 2>&1 || { tail -30 gpurun_out/${TAG}_e2e.log; exit 1; }
cat gpurun_out/${TAG}_e2e.log
