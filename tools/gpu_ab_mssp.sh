# A/B of mssp_kernel knobs: sweeps per workgroup and the fabric_rtt bench line
# per setting of SPF_MSSP_SKIP; usage: TAG=<dir> bash tools/gpu_ab_mssp.sh
set -u
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_mssp.py tests/test_gpu_engine.py tests/test_gpu_fullsize.py -k "mssp or rtt or wan2k or weighted or metric or narrow" -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for a in 0 1; do export SPF_MSSP_SKIP=$a;
  timeout -k 10 200 python -u tools/mssp_stats.py fabric_rtt > $O/stats_a$a.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py --workload fabric_rtt --steps 20 --warmup 3 --cpu-budget 0 > $O/bench_a$a.json 2> $O/bench_a$a.err || exit 1
done
for a in 0 1; do export SPF_MSSP_SKIP=$a; cat $O/stats_a$a.log; python -c "import json,sys; d=json.load(open('$O/bench_a$a.json')); print('ms', d['ms_per_step'], d['roofline'].get('kernel_ms'))"; done
