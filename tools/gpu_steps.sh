#!/bin/bash
# GPU steps (tests, smoke, bench lines, kernel-trace profiles, multi-member
# runs), each under its own time limit, stopping at the first failure;
# outputs under gpurun_out/$TAG.
#   TAG=r06_x STEPS="tests smoke bench prof" WORKLOADS="fabric_full" bash tools/gpu_steps.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r06}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "[$(date +%T)] $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"; tail -4 "$OUT/$name.log"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for s in ${STEPS:-tests}; do
  case $s in
    tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ;;
    ptests) run pytest_sel 900 python -u -m pytest ${PYTEST_FILES} -m gpu --maxfail=15 -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) for w in ${WORKLOADS:-fabric_full}; do
             run bench_$w 400 python -u bench.py --workload $w ${BENCH_ARGS:-}
             grep '^{' "$OUT/bench_$w.log" | tail -1 > "$OUT/bench_$w.json"
           done ;;
    wprof) SPF_WHATIF_PROF=1 SPF_WHATIF_DEBUG=1 run bench_ba_whatif_prof 400 python -u bench.py --workload ba_whatif --steps 2 --warmup 1 --cpu-budget 0 ;;
    gwprof) SPF_WHATIF_PROF=global SPF_WHATIF_DEBUG=1 run bench_ba_whatif_gprof 400 python -u bench.py --workload ba_whatif --steps 2 --warmup 1 --cpu-budget 0 ;;
    gwtests) SPF_WHATIF_PROF=global run pytest_whatif_gprof 900 python -u -m pytest tests/test_gpu_whatif.py "tests/test_gpu_fullsize.py::test_whatif_ba250k_16k_failures_match_oracle" "tests/test_gpu_fullsize.py::test_whatif_ba20k_every_failure_matches_oracle" -m gpu -x -v --timeout 300 --timeout-method thread ;;
    multi) for n in ${MULTI_WORLDS:-2 8}; do
             ids=$(python3 -c "print(','.join(['0']*$n))")
             run multi_x$n 400 python -u bench.py --workload ${MW:-fabric_full} --devices $ids --steps 20 --cpu-budget 0
             grep '^{' "$OUT/multi_x$n.log" | tail -1 > "$OUT/multi_x$n.json"
           done ;;
    prof) for w in ${PROF_WORKLOADS:-fabric_full}; do
            run prof_$w 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv \
              -- python3 -u bench.py --workload $w --steps ${PSTEPS:-5} --warmup 1 --cpu-budget 0
            find "$OUT/prof_$w" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$w.csv" \;
          done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo done
