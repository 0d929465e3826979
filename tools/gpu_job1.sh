#!/bin/bash
# GPU box: quick C2 bench (text cache off / on), the profiling build's region breakdown, SF diag
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 300 python -u bench.py --no-hg19r --no-cpu --check 0 --no-pipeline > gpurun_out/b2.json 2> gpurun_out/b2.err || exit $?
GWA_TEXT_CACHE=1 timeout -k 10 300 python -u bench.py --no-hg19r --no-cpu --check 0 --no-pipeline > gpurun_out/b2tc.json 2> gpurun_out/b2tc.err || exit $?
GWA_LIB=libgwa_prof.so timeout -k 10 300 python -u bench.py --no-hg19r --no-cpu --check 0 --no-pipeline --steps 1 --warmup 0 > gpurun_out/prof.json 2> gpurun_out/prof.err || exit $?
timeout -k 10 400 python -u tools/diag_sf.py 2000 sf,bsf > gpurun_out/diag.log 2>&1
