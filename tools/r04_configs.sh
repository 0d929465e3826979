#!/bin/bash
# GPU box: the full-size config tests (C2/C4 on hg19 and hg19r, C5 pairs, C3 two processes)
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
timeout -k 10 1150 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_configs_hg19.py -m gpu -v --timeout 900 --timeout-method thread --durations=0 > gpurun_out/cfg_tests.log 2>&1
