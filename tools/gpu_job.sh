#!/bin/bash
# GPU box: A/B of the SAM writer's batched text copies (C2) and of the deep-tier LDS queue
# condition (hg19r), then the GPU tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
L=genome-weaver-align_amd
timeout -k 10 400 python -u tools/ab.py --steps 3 $L/libgwa_deep.so $L/libgwa.so > gpurun_out/ab_s2.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab.py --steps 3 --genome hg19r $L/libgwa_deep.so $L/libgwa.so > gpurun_out/ab_sr.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t6.log 2>&1
