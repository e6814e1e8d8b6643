# persistent decode layers vs the launch chain: bench lines (no CPU baseline) for C3 greedy, C2 and C3 beam3
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
for cfg in ${CFGS:-"c3:" "c2:--workload c2" "b3:--decoding beam3"}; do
  name=${cfg%%:*}; args=${cfg#*:}
  for mode in 1 0; do
    ITTS_PL=$mode timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > gpurun_out/bench_${TAG}_${name}_pl$mode.json \
      2> gpurun_out/bench_${TAG}_${name}_pl$mode.err || exit 1
    python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_${name}_pl$mode.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$name PL=$mode', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'])"
  done
done
