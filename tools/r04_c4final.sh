#!/bin/bash
# k >= 4 report threshold 8/16: quick GPU parity, then the C4 -m bsf bench line (parity on every deep-tier read)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests3.log 2>&1 || exit $?
timeout -k 10 400 python3 -u bench.py --workload c4 --no-pipeline > gpurun_out/c4_final.json 2> gpurun_out/c4_final.err
