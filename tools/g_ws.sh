set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_ws}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_mssp.py tests/test_gpu_engine.py tests/test_gpu_fullsize.py tests/test_gpu_linkstate.py tests/test_gpu_multi.py -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; grep -E "FAILED|Error" $O/pytest.log | head -5; [ $rc -ne 0 ] && exit $rc
W=fabric_rtt TAG=${TAG:-r04_ws} CFGS="SPF_WSLICED=1 SPF_WSLICED=0 SPF_WSLICED=1" bash tools/g_env.sh
