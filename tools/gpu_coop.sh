# what-if base pass A/B: cooperative blocks per CU (SPF_COOP_PER_CU)
set -o pipefail
O=gpurun_out/${TAG:-r02_v63}; mkdir -p $O
for k in ${PER_CU:-1 2 4}; do
  SPF_COOP_PER_CU=$k SPF_WHATIF_PROF=1 timeout -k 10 200 python3 -u bench.py --workload ba_whatif --steps 1 --warmup 1 --cpu-budget 0 > $O/prof_$k.log 2>&1 || exit 1
  SPF_COOP_PER_CU=$k timeout -k 10 200 python3 -u bench.py --workload ba_whatif --steps 10 --warmup 2 --cpu-budget 0 > $O/bench_$k.log 2>&1 || exit 1
done
