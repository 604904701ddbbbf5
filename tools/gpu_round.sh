#!/bin/bash
# One GPU session: GPU tests, default bench lines, kernel-trace profile.
#   TAG=r02_v1 bash tools/gpu_round.sh [tests|bench|prof ...]
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
steps="${*:-tests bench prof}"
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; tail -5 "$OUT/pytest_gpu.log"; echo "tests rc=$rc"
      [ $rc -ge 124 ] && exit $rc ;;
    bench)
      for w in ${WORKLOADS:-fabric_full grid100 fabric_rtt}; do
        timeout -k 10 300 python -u bench.py --workload $w ${BENCH_ARGS:-} > "$OUT/bench_$w.log" 2>&1 \
          || { echo "bench $w failed"; tail -20 "$OUT/bench_$w.log"; exit 1; }
        grep '^{' "$OUT/bench_$w.log" | tail -1 > "$OUT/bench_$w.json"; echo "bench $w ok"
      done ;;
    prof)
      for w in ${PROF_WORKLOADS:-fabric_full}; do
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv \
          -- python3 -u bench.py --workload $w --steps ${STEPS:-5} --warmup 1 --cpu-budget 0 \
          > "$OUT/prof_$w.log" 2>&1
        rc=$?; echo "prof $w rc=$rc"; [ $rc -ne 0 ] && { tail -30 "$OUT/prof_$w.log"; exit $rc; }
        find "$OUT/prof_$w" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$w.csv" \;
      done ;;
  esac
done
echo done
