set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in fabric_full grid100 wan_ksp2 ba_whatif; do
  timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -5 gpurun_out/bench_$w.log; exit 1; }
  grep '^{' gpurun_out/bench_$w.log | tail -1 > gpurun_out/bench_$w.json
  echo "bench $w ok"
done
WORKLOADS="fabric_full grid100" PMC=1 bash tools/prof_workloads.sh > gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
for w in fabric_full grid100; do
  python3 tools/pmc_summary.py gpurun_out/pmc_$w --json gpurun_out/pmc_$w.json > gpurun_out/pmc_summary_$w.txt 2>&1 || true
done
# last: the ba_whatif process segfaults in exit-time teardown under rocprofv3
# (after the profiler has written its files; the same with the r01_v13
# library, never without the profiler), so nothing GPU runs after it here --
# its PMC passes go one per gpurun call
WORKLOADS="wan_ksp2 ba_whatif" bash tools/prof_workloads.sh >> gpurun_out/prof.log 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
echo done
