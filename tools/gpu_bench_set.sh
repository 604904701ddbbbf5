# Parity suites + bench lines of a set of workloads (no CPU baseline);
# usage: TAG=<dir> TESTS="tests/..." WL="fabric_full fabric_ref" bash tools/gpu_bench_set.sh
set -u
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for w in ${WL:-fabric_full}; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --cpu-budget 0 > $O/bench_$w.json 2> $O/bench_$w.err || exit 1
  python -c "import json; d=json.load(open('$O/bench_$w.json')); r=d.get('roofline') or {}; print('$w', round(d['ms_per_step'],4), {k: round(v,4) for k,v in (r.get('kernel_ms') or {}).items()})"
done
