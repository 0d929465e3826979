#!/bin/bash
# GPU box: round-end rehearsal on the current tree -- what the driver runs: the GPU tests, smoke(),
# and the default bench line (outputs under gpurun_out/rehearse/)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
D=gpurun_out/rehearse
mkdir -p $D
timeout -k 10 780 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread --durations=15 > $D/tests.log 2>&1 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $D/bench.json 2> $D/bench.err
