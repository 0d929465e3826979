#!/bin/bash
# C4 -m sf: the round-3 tree's bench (bisect/ada8532, its own libgwa.so) for reference, then A/B of
# the round-4 library before (ab_base) and after (ab_cur) the spill fixes, -m sf and -m bsf
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
R=$PWD
(cd bisect/ada8532 && timeout -k 10 300 python3 -u bench.py --workload c4 --strategy sf --no-pipeline --no-cpu --check 0 --steps 3 --warmup 1 > $R/gpurun_out/sfb_ada8532.json 2> $R/gpurun_out/sfb_ada8532.err) || exit $?
timeout -k 10 400 python -u tools/ab.py --workload c4 --strategy sf --genome hg19 --steps 3 tools/ab_base.so tools/ab_cur.so > gpurun_out/ab_sf.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab.py --workload c4 --genome hg19 --steps 3 tools/ab_base.so tools/ab_cur.so > gpurun_out/ab_c4b.log 2>&1
