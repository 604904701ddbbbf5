#!/bin/bash
# PMC passes (one rocprofv3 --pmc pass per counter group, each under its own
# timeout) over short bench runs, summarised per kernel into
# gpurun_out/$TAG/pmc_<workload>.json.
#   TAG=r02_v4 WORKLOADS="fabric_full grid100" bash tools/pmc_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
for w in ${WORKLOADS:-fabric_full}; do
  OUT=gpurun_out/$TAG/pmc_$w
  rm -rf "$OUT"; mkdir -p "$OUT"
  i=0
  while IFS= read -r group; do
    [ -z "$group" ] && continue
    i=$((i+1))
    timeout -k 10 180 rocprofv3 --pmc $group -d "$OUT/p$i" -o run --output-format csv \
      -- python3 -u bench.py --workload $w --steps 2 --warmup 1 --cpu-budget 0 > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "$w pass $i ($group) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
  done <<< "${PMC_GROUPS:-FETCH_SIZE
WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT}"
  python3 tools/pmc_summary.py "$OUT" --json "gpurun_out/$TAG/pmc_$w.json" --source "$TAG" > "$OUT/summary.txt" 2>&1 \
    || { tail -5 "$OUT/summary.txt"; exit 1; }
done
echo done
