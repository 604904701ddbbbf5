# A/B of grouped next-hop units (SPF_SLICED_GROUP) plus the parity suites that
# cover the sliced pass; usage: TAG=<dir> bash tools/gpu_ab_group.sh
set -u
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_team.py tests/test_gpu_sharded.py tests/test_gpu_linkstate.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for gr in 1 0; do
  for w in fabric_full fabric_ref fabric_lfa; do
    SPF_SLICED_GROUP=$gr timeout -k 10 300 python -u bench.py --workload $w --steps 20 --warmup 3 --cpu-budget 0 > $O/bench_${w}_g$gr.json 2> $O/bench_${w}_g$gr.err || exit 1
  done
  SPF_SLICED_GROUP=$gr timeout -k 10 300 python -u tools/emulate_ranks.py --worlds 1,8 > $O/emu_g$gr.log 2>&1 || exit 1
done
for f in $O/bench_*.json; do echo $f; cut -c1-400 $f; done
cut -c1-260 $O/emu_g1.log $O/emu_g0.log
