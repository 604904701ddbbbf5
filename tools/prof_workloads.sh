#!/bin/bash
# rocprofv3 kernel stats (and optional PMC passes) for bench workloads.
#   WORKLOADS="wan_ksp2 ba_whatif" PMC=1 bash tools/prof_workloads.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in ${WORKLOADS:-fabric_full}; do
  rm -rf gpurun_out/prof_$w
  echo "=== $w kernel trace"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$w -o run --output-format csv -- python3 -u bench.py --workload $w --steps ${STEPS:-3} --warmup 1 --cpu-budget 0 > gpurun_out/prof_$w.log 2>&1
  rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/prof_$w.log | tail -1
  [ $rc -ne 0 ] && { tail -20 gpurun_out/prof_$w.log; exit $rc; }
  find gpurun_out/prof_$w -name '*kernel_stats.csv' -exec cp {} gpurun_out/kernel_stats_$w.csv \;
  cut -c1-200 gpurun_out/kernel_stats_$w.csv | head -12
  if [ -n "${PMC:-}" ]; then
    i=0
    for group in "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
      i=$((i+1))
      timeout -k 10 300 rocprofv3 --pmc $group -d gpurun_out/pmc_$w/p$i -o run --output-format csv -- python3 -u bench.py --workload $w --steps 1 --warmup 1 --cpu-budget 0 > gpurun_out/pmc_${w}_p$i.log 2>&1
      rc=$?; echo "pmc $w pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
    done
  fi
done
exit 0
