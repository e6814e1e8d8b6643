# C5 long-form throughput by decode chunk size (rows per decode step)
set -o pipefail
for c in ${CHUNKS:-32 128}; do
  timeout -k 10 240 python3 bench.py --workload c5 --chunk $c --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/c5_$c.json 2> gpurun_out/c5_$c.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/c5_$c.json')); print('chunk $c', d['value'], d['ms_per_step'])"
done
