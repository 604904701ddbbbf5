#!/bin/bash
# A/B of the two BFS kernels: engine parity tests, then grid100 / fabric_full
# bench lines under SPF_MSBFS=planes|masks (and SPF_NARROW for the next-hop
# row width).  Each GPU step has its own timeout; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
for w in grid100 fabric_full; do
  for v in ${VARIANTS:-planes,0 planes,1 masks,0 masks,1}; do
    m=${v%,*}; n=${v#*,}
    SPF_MSBFS=$m SPF_NARROW=$n timeout -k 10 200 python -u bench.py --workload $w --cpu-budget 0 > gpurun_out/ab_${w}_${m}_${n}.log 2>&1 || { echo "bench $w $v failed"; tail -20 gpurun_out/ab_${w}_${m}_${n}.log; exit 1; }
    python3 -c "
import json,sys; d=json.loads([l for l in open('gpurun_out/ab_${w}_${m}_${n}.log') if l.startswith('{')][-1]); r=d['roofline']
print('$w $m narrow=$n', round(d['value']), round(d['ms_per_step'],4), {k: round(x,4) for k,x in r['kernel_ms'].items()})"
  done
done
