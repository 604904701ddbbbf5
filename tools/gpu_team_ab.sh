#!/bin/bash
# Team-BFS session: GPU tests (PYTEST_SEL), per-level stamps of one rank
# share, emulated ranks, world-1 team-size A/B.   TAG=r03_vN bash tools/gpu_team_ab.sh
set -u
export TMPDIR=/tmp
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest ${PYTEST_SEL:-tests/test_gpu_team.py} -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/team_stamps.py --rank 1 > $O/stamps_r1.log 2>&1 || exit 1
for w in ${EMU:-fabric_full}; do
  timeout -k 10 300 python -u tools/emulate_ranks.py --workload $w > $O/emu_$w.log 2>&1 || exit 1
  cat $O/emu_$w.log
done
for G in ${GS:-}; do SPF_MSBFS_TEAM=$G timeout -k 10 300 python -u tools/emulate_ranks.py --worlds 1 > $O/emu_w1_G$G.log 2>&1 || exit 1; cat $O/emu_w1_G$G.log; done
