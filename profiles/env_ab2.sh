# C3 decode step per environment setting (HIP events), interleaved twice: ENVS="A=1 A=2"
set -o pipefail
for rep in 1 2; do
for e in ${ENVS}; do
  env $e timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$e', d['roofline']['avg_launch_us'], d['value'])"
done
done
