#!/bin/bash
# A/B timing of library builds on the hg19-size C2 workload (GPU box): tools/ab.sh libA.so libB.so ...
# each library in its own process, alternating twice, one line per run (tools/knob_sweep.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
for rep in 1 2; do
  for v in "$@"; do
    GWA_LIB=$v timeout -k 10 300 python -u tools/knob_sweep.py --var AB_LIB $v --steps 3 2>&1 | grep AB_LIB || exit 1
  done
done
