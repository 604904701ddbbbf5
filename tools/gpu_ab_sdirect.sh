set -u
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_team.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/team_stamps.py --rank 1 > $O/stamps_r1.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/emulate_ranks.py --worlds 1,2,4,8 > $O/emu.log 2>&1 || exit 1
SPF_SDIRECT=0 timeout -k 10 300 python -u tools/emulate_ranks.py --worlds 2,4,8 > $O/emu_nosd.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/emulate_ranks.py --workload grid100 --worlds 1 > $O/emu_grid.log 2>&1 || exit 1
cut -c1-260 $O/emu.log $O/emu_nosd.log $O/emu_grid.log
