#!/bin/bash
# quick GPU parity, C4 -m bsf with the k >= 4 hit lists + last-tier jump, hg19r C4 -m sf
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/knob_sweep.py --genome hg19 --c4 --k 5 --reads 1000000 --steps 2 --var multi \
  "GWA_TIER_JUMP=1" "GWA_TIER_JUMP=0" "GWA_VERIFY_MEMO=0" > gpurun_out/sweep_c4b.log 2>&1 || exit $?
GWA_VERBOSE=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -k "hg19r_indels_k5" --timeout 450 --timeout-method thread > gpurun_out/c4_hg19r.log 2>&1
