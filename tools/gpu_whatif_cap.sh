# what-if A/B: wave-team |D| cap (SPF_WHATIF_WAVECAP) x classify threshold (SPF_WHATIF_CLASSIFY)
set -o pipefail
O=gpurun_out/${TAG:-r02_v60}; mkdir -p $O
for v in ${VARIANTS:-1024:1024 2048:1024 2048:2048 4096:1024 1024:512}; do
  SPF_WHATIF_WAVECAP=${v%%:*} SPF_WHATIF_CLASSIFY=${v##*:} timeout -k 10 200 python3 -u bench.py --workload ba_whatif --steps 10 --warmup 2 --cpu-budget 0 > $O/whatif_${v/:/_}.log 2>&1 || exit 1
done
