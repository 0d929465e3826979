#!/bin/bash
# Kernel-trace + PMC profiles of bench.py on the GPU box (run through gpurun).
# usage: [PASS=all|trace|pmc] tools/profile.sh <tag> [bench args...]
#   trace: rocprofv3 --kernel-trace --stats of the full bench command
#   pmc:   four separate counter passes (FETCH_SIZE; SQ_*; TCC hit/miss; WRITE_SIZE) of the timed leg only
set -o pipefail
TAG=$1; shift
ARGS="$@"
PASS=${PASS:-all}
cd "${GRAFT_REPO_ROOT:-$(dirname $0)/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
if [ "$PASS" = all ] || [ "$PASS" = trace ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -- python3 bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err || exit $?
fi
if [ "$PASS" = all ] || [ "$PASS" = pmc ]; then
  LEG="--no-cpu --check 0 --no-pipeline --no-hg19r"
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T --output-format csv -d $OUT/pmc_fetch -- python3 bench.py $ARGS $LEG > $OUT/bench_pmc1.json 2> $OUT/pmc1.err || exit $?
  timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --kernel-trace -T --output-format csv -d $OUT/pmc_sq -- python3 bench.py $ARGS $LEG > $OUT/bench_pmc2.json 2> $OUT/pmc2.err || exit $?
  timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace -T --output-format csv -d $OUT/pmc_tcc -- python3 bench.py $ARGS $LEG > $OUT/bench_pmc3.json 2> $OUT/pmc3.err || exit $?
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T --output-format csv -d $OUT/pmc_write -- python3 bench.py $ARGS $LEG > $OUT/bench_pmc4.json 2> $OUT/pmc4.err || exit $?
fi
find $OUT -name "*.csv" | head -50 > $OUT/files.txt
