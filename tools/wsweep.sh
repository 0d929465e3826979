# report-batching threshold sweep (GWA_WAITQ16) on the 200 Mbp / 1M-read workload (GPU box)
set -o pipefail
for q in "$@"; do
  GWA_WAITQ16=$q timeout -k 10 300 python bench.py --genome 200 --reads 1000000 --steps 3 --warmup 1 --no-cpu --check 200 > gpurun_out/bq_$q.json 2> gpurun_out/bq_$q.err || exit 1
done
