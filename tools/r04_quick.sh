#!/bin/bash
# GPU box: quick parity tests (HIP path vs oracle, CLI) then a short C2 bench and a quick-scan order sweep;
# each step time-limited, chained so that a failure ends the call
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/q_tests.log 2>&1 || exit $?
timeout -k 10 420 python -u bench.py --no-cpu --no-pipeline --steps 3 --warmup 1 > gpurun_out/q_bench.json 2> gpurun_out/q_bench.err || exit $?
timeout -k 10 420 python -u tools/knob_sweep.py --genome hg19 --var GWA_QS_SORT 0 16 28 > gpurun_out/q_qs.log 2>&1
