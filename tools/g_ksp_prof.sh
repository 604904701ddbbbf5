set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_k2}; mkdir -p $O
P=${PROF-1}
[ -n "$P" ] && export SPF_KSP2_PROF=$P
for cfg in ${CFGS:-"SPF_KSP2_U16=1" "SPF_KSP2_U16=0"}; do
  tag=$(echo $cfg | tr ' =' '__')
  env $cfg timeout -k 10 300 python -u bench.py --workload wan_ksp2 --cpu-budget 0 --steps ${KSTEPS:-3} --warmup 1 > $O/prof_$tag.log 2>&1 || exit $?
  echo "== $cfg"; grep "ksp2 p" $O/prof_$tag.log | tail -2
  grep '^{' $O/prof_$tag.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(round(d['ms_per_step'],3),d['roofline']['kernel_ms'],d['parity']['mismatches'])"
done
