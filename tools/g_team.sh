#!/bin/bash
# Team-BFS A/B on one box: team tests, rank stamps, single-process x2 / x8 members.
#   TAG=r05_t3 bash tools/g_team.sh
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-team}
mkdir -p "$OUT"
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_team.py ${EXTRA_TESTS:-} -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 300 python -u tools/team_stamps.py --world 8 --rank 1 > "$OUT/stamps.log" 2>&1 || { tail "$OUT/stamps.log"; exit 1; }
head -30 "$OUT/stamps.log"
for n in ${WORLDS:-8 2}; do
  ids=$(python3 -c "print(','.join(['0']*$n))")
  timeout -k 10 300 python -u bench.py --workload fabric_full --devices $ids --steps 20 --cpu-budget 0 > "$OUT/x$n.log" 2>&1 || { tail "$OUT/x$n.log"; exit 1; }
  python3 -c "import json;d=[json.loads(l) for l in open('$OUT/x$n.log') if l.startswith('{')][-1];print('x$n', [round(x,4) for x in d['config']['member_execute_ms']], 'mismatches', d['parity']['mismatches'])"
done
