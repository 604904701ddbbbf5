#!/bin/bash
# A/B experiments: one bench run per environment setting (diagnostics).
#   EXPS="A=1 B=2" WL=fabric_full TAG=x bash tools/gpu_exp.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-exp}; mkdir -p $O
for e in base ${EXPS:-}; do
  if [ "$e" = base ]; then envs=""; else envs="$e"; fi
  env $envs timeout -k 10 200 python -u bench.py --workload ${WL:-fabric_full} --cpu-budget 0 > $O/bench_${e}.log 2>&1 || { tail -5 $O/bench_${e}.log; exit 1; }
  echo "$e: $(grep '^{' $O/bench_${e}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],4), {k: round(v,4) for k,v in d["roofline"]["kernel_ms"].items()})')"
done
for e in ${STAMPS:-}; do
  env $e timeout -k 10 200 python -u tools/stamps.py ${STAMP_WL:-fabric} > $O/stamps_${e}.log 2>&1 || { tail -5 $O/stamps_${e}.log; exit 1; }
  echo "== stamps $e"; cat $O/stamps_${e}.log | grep -v amdgpu.ids
done
