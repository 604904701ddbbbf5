set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_w1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_whatif.py tests/test_gpu_fullsize.py -k "whatif or what_if" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-"SPF_WHATIF_OVF_GROUP=1" "SPF_WHATIF_OVF_GROUP=0"}; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python -u bench.py --workload ba_whatif --cpu-budget 0 > $O/bench_$tag.log 2>&1 || exit $?
  grep '^{' $O/bench_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg',round(d['ms_per_step'],3),d['roofline']['kernel_ms'],d['parity']['mismatches'])"
done
