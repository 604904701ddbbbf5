#!/bin/bash
# mssp A/B: per-sweep statistics and fabric_rtt bench lines under env variants.
#   TAG=r05_ms2 VARIANTS="SPF_MSSP_PHASED=0 SPF_MSSP_PHASED=1" bash tools/g_ms.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-ms}
mkdir -p "$OUT"
for v in ${VARIANTS:-SPF_MSSP_PHASED=0}; do
  env $v timeout -k 10 200 python -u tools/mssp_stats.py fabric_rtt > "$OUT/stats_$v.log" 2>&1 || { tail "$OUT/stats_$v.log"; exit 1; }
  env $v timeout -k 10 300 python -u bench.py --workload fabric_rtt --steps 10 --warmup 2 --cpu-budget 0 > "$OUT/bench_$v.log" 2>&1 || { tail "$OUT/bench_$v.log"; exit 1; }
  python3 -c "import json;d=[json.loads(l) for l in open('$OUT/bench_$v.log') if l.startswith('{')][-1];print('$v', round(d['ms_per_step'],4), d['roofline'].get('kernel_ms'), d['parity'])"
  grep "sweeps total\|per sweep" "$OUT/stats_$v.log"
done
