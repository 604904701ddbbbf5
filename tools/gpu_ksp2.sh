#!/bin/bash
# KSP2 bring-up: GPU parity tests for the batched KSP2 kernel, then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_ksp2.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ksp2_tests.log 2>&1
rc=$?; tail -15 gpurun_out/ksp2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --workload wan_ksp2 --steps 3 --warmup 1 --cpu-budget 10 > gpurun_out/ksp2_bench.log 2>&1
rc=$?; tail -3 gpurun_out/ksp2_bench.log; exit $rc
