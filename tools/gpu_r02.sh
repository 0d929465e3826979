#!/bin/bash
# GPU-box check of this round's work: gpu tests, a 2-rank bench on one GPU, the default bench.
set -o pipefail
TAG=${1:-r02}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>/dev/null; } > gpurun_out/${TAG}_host.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u bench.py --gpus 2 --genome 200 --reads 2000000 --steps 2 --no-cpu --check 5000 --no-pipeline > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { tail -30 gpurun_out/${TAG}_bench2.err; exit 1; }
cat gpurun_out/${TAG}_bench2.json
timeout -k 10 900 python -u bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
