set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02_v23; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_whatif.py -v --timeout 300 --timeout-method thread > $O/pytest_whatif.log 2>&1; rc=$?; tail -12 $O/pytest_whatif.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --workload fabric_full --cpu-budget 0 > $O/bench_fabric_full.log 2>&1 || exit 1
tail -3 $O/bench_fabric_full.log
SPF_WHATIF_PROF=1 timeout -k 10 200 python -u bench.py --workload ba_whatif --steps 1 --warmup 1 --cpu-budget 0 > $O/whatif_prof.log 2>&1 || exit 1
TAG=r02_v23 WORKLOADS="fabric_full grid100" bash tools/pmc_round.sh
