#!/bin/bash
# A/B of tools/ab_base.so vs tools/ab_new.so (C2 hg19, then C4), SAM compared
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
timeout -k 10 500 python -u tools/ab.py --workload c2 --genome hg19 --steps 4 tools/ab_base.so tools/ab_new.so tools/ab_new2.so > gpurun_out/ab_r04.log 2>&1 || exit $?
timeout -k 10 500 python -u tools/ab.py --workload c4 --genome hg19 --steps 3 tools/ab_base.so tools/ab_new.so tools/ab_new2.so > gpurun_out/ab_r04_c4.log 2>&1
