#!/bin/bash
# One gpurun call: smoke -> GPU parity tests -> bench -> rocprofv3 kernel stats.
# Every GPU step runs under its own timeout; a crash/timeout (rc not 0/1) stops
# the script so nothing else touches the GPU after a fault.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p "$OUT"
STEPS="${STEPS:-smoke,tests,bench,prof}"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $* ($(date +%T))"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  tail -n 8 "$OUT/$name.log"
  return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
has() { [[ ",$STEPS," == *",$1,"* ]]; }
if has smoke; then
  run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?
  fatal $rc && exit $rc
fi
if has tests; then
  run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}; rc=$?
  fatal $rc && exit $rc
fi
if has bench; then
  run bench 400 python -u bench.py ${BENCH_ARGS:-}; rc=$?
  fatal $rc && exit $rc
  grep '^{' "$OUT/bench.log" | tail -1 > "$OUT/bench.json"
fi
if has prof; then
  rm -rf "$OUT/prof"
  run rocprof 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 -u bench.py --steps 5 --warmup 1 --cpu-budget 0 ${BENCH_ARGS:-}; rc=$?
  fatal $rc && exit $rc
  find "$OUT/prof" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
  cat "$OUT/kernel_stats.csv" 2>/dev/null | head -20
fi
exit 0
