#!/bin/bash
# Round-4 GPU session: GPU tests, emulated ranks, bench lines, a ba_whatif
# kernel trace (grid-resident launches instead of cooperative ones).
#   TAG=r03_v2 STEPS="tests emulate bench trace" bash tools/gpu_r04.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for s in ${STEPS:-tests emulate bench trace}; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -v --timeout 300 --timeout-method thread \
        ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
      rc=$?; tail -5 "$OUT/pytest_gpu.log"; echo "tests rc=$rc"
      [ $rc -ne 0 ] && exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
      rc=$?; tail -3 "$OUT/smoke.log"; [ $rc -ne 0 ] && exit $rc ;;
    emulate)
      for w in ${EMU_WORKLOADS:-fabric_full grid100 fabric_rtt}; do
        timeout -k 10 300 python -u tools/emulate_ranks.py --workload $w > "$OUT/emulate_$w.log" 2>&1
        rc=$?; cat "$OUT/emulate_$w.log" | grep '^{' ; [ $rc -ne 0 ] && { tail -20 "$OUT/emulate_$w.log"; exit $rc; }
      done ;;
    bench)
      for w in ${WORKLOADS:-fabric_full grid100 fabric_rtt}; do
        timeout -k 10 300 python -u bench.py --workload $w ${BENCH_ARGS:-} > "$OUT/bench_$w.log" 2>&1
        rc=$?; [ $rc -ne 0 ] && { echo "bench $w failed rc=$rc"; tail -20 "$OUT/bench_$w.log"; exit $rc; }
        grep '^{' "$OUT/bench_$w.log" | tail -1 > "$OUT/bench_$w.json"; echo "bench $w ok"
      done ;;
    multi)
      # single-process multi-device context, members on one GPU (emulated N)
      for w in ${MULTI_WORKLOADS:-fabric_full}; do
        for n in ${MULTI_WORLDS:-2 4 8}; do
          ids=$(python3 -c "print(','.join(['0']*$n))")
          for gflag in "" ${MULTI_GRAPHS:---graphs}; do
            tagm=${w}_x${n}${gflag:+_graphs}
            timeout -k 10 300 python -u bench.py --workload $w --devices $ids $gflag --steps ${MSTEPS:-20} \
              > "$OUT/multi_$tagm.log" 2>&1
            rc=$?; [ $rc -ne 0 ] && { echo "multi $tagm failed rc=$rc"; tail -20 "$OUT/multi_$tagm.log"; exit $rc; }
            grep '^{' "$OUT/multi_$tagm.log" | tail -1 > "$OUT/multi_$tagm.json"
            python3 -c "import json;d=json.load(open('$OUT/multi_$tagm.json'));c=d['config'];print('multi $tagm', round(d['ms_per_step'],4), [round(x,4) for x in c['member_execute_ms']], d['parity']['mismatches'])"
          done
        done
      done ;;
    prof)
      for w in ${PROF_WORKLOADS:-fabric_full}; do
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$w" -o run --output-format csv \
          -- python3 -u bench.py --workload $w --steps ${PSTEPS:-5} --warmup 1 --cpu-budget 0 \
          > "$OUT/prof_$w.log" 2>&1
        rc=$?; echo "prof $w rc=$rc"; [ $rc -ne 0 ] && { tail -30 "$OUT/prof_$w.log"; exit $rc; }
        find "$OUT/prof_$w" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats_$w.csv" \;
      done ;;
    trace)
      PROF_WORKLOADS=ba_whatif PSTEPS=3 STEPS=prof bash tools/gpu_r04.sh || exit $? ;;
    pmc)
      TAG=$TAG WORKLOADS="${PMC_WORKLOADS:-fabric_full}" bash tools/pmc_round.sh || exit $? ;;
  esac
done
echo done
