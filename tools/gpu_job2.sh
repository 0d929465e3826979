#!/bin/bash
# GPU box: quick C2 bench, C4 -m bsf bench with parity (hybrid heap)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 300 python -u bench.py --no-hg19r --no-cpu --check 0 --no-pipeline > gpurun_out/b3.json 2> gpurun_out/b3.err || exit $?
timeout -k 10 500 python -u bench.py --workload c4 --no-cpu --no-pipeline > gpurun_out/b3c4.json 2> gpurun_out/b3c4.err
