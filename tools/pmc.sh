#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 --pmc pass per counter group,
# each under its own timeout, as MI355X_MICROARCH.md's rocprofv3 section asks).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
rm -rf "$OUT"; mkdir -p "$OUT"
ARGS="--steps 2 --warmup 1 --cpu-budget 0 ${BENCH_ARGS:-}"
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
while IFS= read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  echo "=== pass $i: $group"
  timeout -k 10 120 rocprofv3 --pmc $group -d "$OUT/p$i" -o run --output-format csv -- python3 -u bench.py $ARGS > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<< "${PMC_GROUPS:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT}"
find "$OUT" -name '*counter_collection.csv' | sort
