#!/bin/bash
# GPU-box: end-to-end CLI timing variants (FASTQ -> SAM file, hg19-size index from a saved index).
set -o pipefail
TAG=${1:-e2e}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_cli.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "cli or pipeline or saved or bd" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for cfg in "2 1048576" "4 1048576"; do
set -- $cfg
timeout -k 10 400 python -u tools/e2e_cli.py --reads 16000000 --saved-index --workers $1 --batch $2 > gpurun_out/${TAG}_w$1_b$2.log 2>&1 || { tail -30 gpurun_out/${TAG}_w$1_b$2.log; exit 1; }
cat gpurun_out/${TAG}_w$1_b$2.log
done
