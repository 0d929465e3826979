#!/bin/bash
# GPU box: the profiling build's per-region wavefront cycles (GWA_PROF) for C2 and C4 -m bsf
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
GWA_LIB=libgwa_prof.so timeout -k 10 300 python -u bench.py --no-hg19r --no-cpu --check 0 --no-pipeline --steps 1 --warmup 0 > gpurun_out/prof_c2.json 2> gpurun_out/prof_c2.err || exit $?
GWA_LIB=libgwa_prof.so timeout -k 10 300 python -u bench.py --workload c4 --no-cpu --check 0 --no-pipeline --steps 1 --warmup 0 > gpurun_out/prof_c4.json 2> gpurun_out/prof_c4.err
