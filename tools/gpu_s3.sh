#!/bin/bash
# GPU-box: gpu parity tests, the default bench line, then C4 -m bsf (tier times) into gpurun_out/<tag>_*.
set -o pipefail
TAG=${1:-s3}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cut -c1-600 gpurun_out/${TAG}_bench.json
timeout -k 10 400 python -u bench.py --workload c4 --no-pipeline --no-cpu --check 2000 > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || { tail -30 gpurun_out/${TAG}_c4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_c4.json'));print(d['value'], d['detail'].get('tier_reads'), d['detail'].get('tier_ms'))"
