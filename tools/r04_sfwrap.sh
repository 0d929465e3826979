#!/bin/bash
# quick GPU parity on the current library, then -m sf A/B: ab_cur (spill fixes) vs ab_new (+ WRAP instances)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab.py --workload c4 --strategy sf --genome hg19 --steps 3 tools/ab_cur.so tools/ab_new.so > gpurun_out/ab_sf2.log 2>&1
