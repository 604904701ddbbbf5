# BFS-kernel experiment: parity tests on the BFS kernels, then per-workload
# A/B against the HEAD library (openr_amd/lib/ab/lib_head.so).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${TAG:-pl}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_engine.py tests/test_gpu_fullsize.py -k "${K:-planes or masks or grid or ring or unit or fabric}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for w in ${WS:-grid100}; do
  W=$w ALT=openr_amd/lib/ab/lib_head.so TAG=${TAG:-pl}/$w ROUNDS="1 2 3" bash tools/g_ab.sh || exit $?
done
