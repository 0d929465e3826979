#!/bin/bash
# compiler-option variants of the -m sf children-loop flag form: the 400-bp -m sf GPU
# test against each libgwa_fv_<v>.so; stops at the first run that ends other than pass / test failure
mkdir -p gpurun_out/fv
for v in "$@"; do
  GWA_LIB=libgwa_fv_$v.so timeout -k 10 200 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "long_reads_on_gpu and 400" > gpurun_out/fv/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc" | tee -a gpurun_out/fv/summary.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
