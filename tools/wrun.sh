# A/B timing of library variants on the 200 Mbp / 1M-read workload (GPU box)
set -o pipefail
for v in "$@"; do
  GWA_LIB=$v timeout -k 10 300 python bench.py --genome 200 --reads 1000000 --steps 3 --warmup 1 --no-cpu --check 2000 > gpurun_out/bw_$v.json 2> gpurun_out/bw_$v.err || exit 1
done
