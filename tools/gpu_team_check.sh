# Team BFS check: parity suites that run it, then emulated ranks of the
# fabric split (world 1, 2, 4, 8); usage: TAG=<dir> bash tools/gpu_team_check.sh
set -u
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_team.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/emulate_ranks.py --worlds 1,2,4,8 > $O/emu.log 2>&1 || exit 1
cut -c1-330 $O/emu.log
