set -o pipefail
for v in libgwa.so libgwa_w2.so libgwa_w3.so libgwa_w4.so; do
  GWA_LIB=$v timeout -k 10 100 python tools/dbg_rep.py > gpurun_out/dbg_$v.log 2>&1 || exit 1
  GWA_LIB=$v timeout -k 10 300 python bench.py --genome 200 --reads 1000000 --steps 3 --warmup 1 --no-cpu --check 2000 > gpurun_out/bw_$v.json 2> gpurun_out/bw_$v.err || exit 1
done
