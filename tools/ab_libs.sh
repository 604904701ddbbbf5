#!/bin/bash
# Bench the same workload against alternative in-tree builds
# (openr_amd/lib/variants/lib_<v>.so, OPENR_SPF_LIB) -- kernel experiments.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
W=${W:-grid100}
for v in ${LIBS:-A B C}; do
  OPENR_SPF_LIB=openr_amd/lib/variants/lib_$v.so timeout -k 10 200 python -u bench.py --workload $W --cpu-budget 0 --steps 10 > gpurun_out/ablib_$v.log 2>&1 || { tail -20 gpurun_out/ablib_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('gpurun_out/ablib_$v.log') if l.startswith('{')][-1]); print('lib $v', d['roofline']['kernel_ms'])"
done
