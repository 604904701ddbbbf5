#!/bin/bash
# What-if bring-up: GPU parity tests, then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_whatif.py -x -v --timeout 400 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/whatif_tests.log 2>&1
rc=$?; tail -15 gpurun_out/whatif_tests.log; [ $rc -ne 0 ] && exit $rc
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 300 python -u bench.py --workload ba_whatif --steps 3 --warmup 1 --cpu-budget 10 > gpurun_out/whatif_bench.log 2>&1
rc=$?; tail -3 gpurun_out/whatif_bench.log; exit $rc
