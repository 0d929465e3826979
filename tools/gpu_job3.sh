#!/bin/bash
# GPU box: A/B of libgwa builds on C2, then the C4 -m bsf line
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 400 python -u tools/ab.py --steps 3 genome-weaver-align_amd/libgwa.so genome-weaver-align_amd/libgwa_pick.so > gpurun_out/ab1.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --workload c4 --no-cpu --check 0 --no-pipeline > gpurun_out/b4c4.json 2> gpurun_out/b4c4.err
