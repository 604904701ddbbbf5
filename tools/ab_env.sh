#!/bin/bash
# A/B a knob: the same bench workload under several environment settings.
#   VAR=SPF_ECMP_BPC VALUES="0 2 4 6 8" WORKLOAD=fabric_full TAG=x bash tools/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
for v in $VALUES; do
  for w in ${WORKLOAD:-fabric_full}; do
    env "$VAR=$v" timeout -k 10 200 python -u bench.py --workload $w --steps ${STEPS:-50} --warmup 5 --cpu-budget 0 > "$OUT/${w}_${VAR}_$v.log" 2>&1 || { echo "fail $w $v"; tail -5 "$OUT/${w}_${VAR}_$v.log"; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],4), {k: round(v,4) for k,v in d['roofline']['kernel_ms'].items()})" "$OUT/${w}_${VAR}_$v.log" "$w" "$VAR=$v"
  done
done
