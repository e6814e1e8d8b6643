# persistent decode layer: bit-identity vs the launch chain, then C3 bench with the persistent layers
# (default) and with the launch chain (ITTS_PL=0)
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/pl_test_$TAG.txt 2>&1
rc=$?; tail -12 gpurun_out/pl_test_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for mode in 1 0; do
  ITTS_PL=$mode timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_${TAG}_pl$mode.json \
    2> gpurun_out/bench_${TAG}_pl$mode.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_pl$mode.json').read().strip().splitlines()[-1]);r=d['roofline'];print('PL=$mode', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'])"
done
