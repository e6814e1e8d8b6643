# decode step per environment variant (HIP events, bench.py 3 steps), interleaved twice:
#   VARIANTS="base ITTS_PL_KEEP_LAYERS=6 ..." (base = no extra env), ARGS = extra bench args
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${VARIANTS:-base}; do
  if [ "$v" = base ]; then envs=""; else envs="$v"; fi
  env $envs timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 $ARGS > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$v', d['roofline']['avg_launch_us'], d['value'])"
done
done
