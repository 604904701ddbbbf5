# KSP2 A/B: k = 2 SPF bucket width (SPF_KSP2_DELTA) x sources per workgroup (SPF_KSP2_CHUNK)
set -o pipefail
O=gpurun_out/${TAG:-r02_v49}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_ksp2.py tests/test_gpu_fullsize.py tests/test_gpu_sr_routes.py -m gpu -x -q --timeout 300 --timeout-method thread -k "ksp2 or kth or KSP or sr" > $O/pytest.log 2>&1 || exit 1
for c in ${CHUNKS:-64 512 2048}; do for d in ${DELTAS:-4294967295 default 125}; do
  if [ $d = default ]; then unset SPF_KSP2_DELTA; else export SPF_KSP2_DELTA=$d; fi
  SPF_KSP2_CHUNK=$c timeout -k 10 200 python3 -u bench.py --workload wan_ksp2 --steps 3 --warmup 1 --cpu-budget 0 > $O/ksp2_c${c}_d$d.log 2>&1 || exit 1
done; done
