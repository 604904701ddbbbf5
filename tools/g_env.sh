# Env-knob sweep of one workload on one box:
#   W=ba_whatif CFGS="SPF_WHATIF_GROUP=4 SPF_WHATIF_GROUP=8" TAG=x bash tools/g_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-env}; mkdir -p $O
for cfg in $CFGS; do
  tag=$(echo $cfg | tr ' =,' '___')
  env $(echo $cfg | tr ',' ' ') timeout -k 10 ${TMO:-200} python -u bench.py --workload $W --cpu-budget 0 ${BENCH_ARGS:-} > $O/$tag.log 2>&1 || { echo "$cfg failed"; tail -3 $O/$tag.log; exit 1; }
  grep '^{' $O/$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg',round(d['ms_per_step'],4),{k:round(v,4) for k,v in d['roofline']['kernel_ms'].items()},d.get('parity',{}).get('mismatches'))"
done
