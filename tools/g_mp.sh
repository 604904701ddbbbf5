set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_m1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_mssp.py tests/test_gpu_fullsize.py -k "mssp or rtt" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-"X=1"}; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python -u bench.py --workload fabric_rtt --cpu-budget 0 > $O/bench_$tag.log 2>&1 || exit $?
  grep '^{' $O/bench_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg',round(d['ms_per_step'],4),{k:round(v,4) for k,v in d['roofline']['kernel_ms'].items()},d['parity']['mismatches'])"
done
