#!/bin/bash
# quick GPU parity + CLI tests on the current library (incl. the short-read / large-k -m sf instance test)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/q_tests2.log 2>&1
