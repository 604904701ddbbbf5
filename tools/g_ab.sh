# A/B of one workload between the in-tree library and an alternative build
# (OPENR_SPF_LIB), alternating runs on one box.
#   W=fabric_rtt ALT=openr_amd/lib/ab/libopenr_spf_mssp_old.so TAG=x bash tools/g_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}; mkdir -p $O
for r in ${ROUNDS:-1 2}; do
  for v in new alt; do
    if [ $v = alt ]; then export OPENR_SPF_LIB=$ALT; else unset OPENR_SPF_LIB; fi
    timeout -k 10 300 python -u bench.py --workload $W --cpu-budget 0 ${BENCH_ARGS:-} > $O/${v}_$r.log 2>&1 || exit $?
    grep '^{' $O/${v}_$r.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$v $r',round(d['ms_per_step'],4),{k:round(v,4) for k,v in d['roofline']['kernel_ms'].items()},d.get('parity',{}).get('mismatches'))"
  done
done
