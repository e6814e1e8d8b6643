# bench A/B of an environment switch: ENVS="A=1 A=0 ..." (decode us per replay, audio-s/s)
set -o pipefail
for e in ${ENVS}; do
  env $e timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$e', d['roofline']['avg_launch_us'], d['value'])"
done
