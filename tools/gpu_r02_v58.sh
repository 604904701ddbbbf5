# round refresh after the KSP2 changes: every GPU test, every bench line,
# kernel stats of wan_ksp2 and fabric_full, PMC passes of wan_ksp2
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
TAG=r02_v58 WORKLOADS="fabric_full grid100 fabric_rtt fabric_ref wan_ksp2 ba_whatif fabric_lfa" PROF_WORKLOADS="wan_ksp2 fabric_full" bash tools/gpu_round.sh tests bench prof || exit $?
grep -q " passed" gpurun_out/r02_v58/pytest_gpu.log && ! grep -q " failed" gpurun_out/r02_v58/pytest_gpu.log || exit 1
TAG=r02_v58 WORKLOADS="wan_ksp2" bash tools/pmc_round.sh
