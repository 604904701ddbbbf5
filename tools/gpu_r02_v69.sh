# end-of-session refresh: every bench line, kernel stats (fabric_full, wan_ksp2),
# PMC of fabric_full; the ba_whatif kernel trace last (exit fault)
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=r02_v69 WORKLOADS="fabric_full grid100 fabric_rtt fabric_ref wan_ksp2 ba_whatif fabric_lfa" PROF_WORKLOADS="fabric_full wan_ksp2" bash tools/gpu_round.sh bench prof || exit $?
TAG=r02_v69 WORKLOADS="fabric_full" bash tools/pmc_round.sh || exit $?
O=gpurun_out/r02_v69
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ba_whatif -o run --output-format csv -- python3 -u bench.py --workload ba_whatif --steps 5 --warmup 1 --cpu-budget 0 > $O/prof_ba_whatif.log 2>&1
echo "ba_whatif trace rc=$?"
find $O/prof_ba_whatif -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_ba_whatif.csv \;
exit 0
