set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_k1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ksp2_compact.py tests/test_gpu_ksp2.py tests/test_gpu_fullsize.py -k "ksp2 or compact" -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -15 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload wan_ksp2 --cpu-budget 0 > $O/bench16.log 2>&1 || exit $?
SPF_KSP2_U16=0 timeout -k 10 300 python -u bench.py --workload wan_ksp2 --cpu-budget 0 > $O/bench32.log 2>&1 || exit $?
for f in bench16 bench32; do grep '^{' $O/$f.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$f',round(d['ms_per_step'],3),d['roofline']['kernel_ms'],d['parity']['mismatches'])"; done
