# attn.c_proj in the decode chain: split-K 8 + reduce (default) vs one 16-column residual-epilogue launch
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
for rep in 1 2; do
for mode in 0 1; do
  ITTS_PL=0 ITTS_OPROJ_EPI=$mode timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 > gpurun_out/oproj_${TAG}_$mode.json 2> gpurun_out/oproj_${TAG}_$mode.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/oproj_${TAG}_$mode.json').read().strip().splitlines()[-1]);r=d['roofline'];print('OPROJ_EPI=$mode', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'])"
done
done
