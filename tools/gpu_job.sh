#!/bin/bash
# GPU box: profiling-build region breakdown (C2, C4 -m bsf), A/B of the baseline and current
# library on C4 -m bsf, then the GPU test suite
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
Q="--no-hg19r --no-cpu --check 0 --no-pipeline"
L=genome-weaver-align_amd
GWA_LIB=libgwa_prof.so timeout -k 10 300 python -u bench.py $Q --steps 1 --warmup 0 > gpurun_out/p_c2.json 2> gpurun_out/p_c2.err || exit $?
GWA_LIB=libgwa_prof.so timeout -k 10 400 python -u bench.py $Q --workload c4 --steps 1 --warmup 0 > gpurun_out/p_c4.json 2> gpurun_out/p_c4.err || exit $?
timeout -k 10 400 python -u tools/ab.py --workload c4 --steps 2 $L/libgwa_base.so $L/libgwa.so > gpurun_out/ab_c4.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t2.log 2>&1
