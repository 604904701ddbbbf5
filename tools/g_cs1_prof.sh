#!/bin/bash
# CS-1 (fabric_lfa_routes) host-side profile: cProfile over the bench, then
# the cumulative / self-time tables of everything under buildRouteDb.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05_cs1}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m cProfile -o "$OUT/cs1.prof" bench.py --workload fabric_lfa_routes \
  --steps ${STEPS:-5} --warmup 1 --cpu-budget 0 > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 1; }
python - "$OUT" <<'PY'
import pstats, sys
out = sys.argv[1]
with open(f"{out}/stats.txt", "w") as f:
    st = pstats.Stats(f"{out}/cs1.prof", stream=f)
    st.sort_stats("cumulative").print_stats(60)
    st.sort_stats("tottime").print_stats(40)
PY
grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
echo done
