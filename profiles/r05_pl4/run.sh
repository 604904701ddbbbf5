set -e
mkdir -p gpurun_out/r05_pl4
for v in 0 1 3 0 1; do
  SPF_PLANES4=$v timeout -k 10 180 python -u bench.py --workload grid100 --steps 20 --warmup 3 --cpu-budget 0 > gpurun_out/r05_pl4/grid100_p$v.json 2> gpurun_out/r05_pl4/grid100_p$v.err
  echo "p$v: $(python -c "import json,sys;d=json.loads(open('gpurun_out/r05_pl4/grid100_p$v.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d.get('parity'), d.get('kernels', '')) ")"
done
