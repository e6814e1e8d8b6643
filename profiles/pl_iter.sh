# persistent-layer iteration: bit-identity tests, the C3-shaped phase trace, C3 / C2 bench lines
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py tests/test_gpu_longform.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_test_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/pl_test_$TAG.txt; [ $rc -eq 0 ] || exit $rc
STEPS=200 ITTS_HIP_LIB=$PWD/index-tts-dubbing_amd/indextts/libitts_hip_trace.so timeout -k 10 200 python -u profiles/pl_trace.py 32 > gpurun_out/pl_trace_$TAG.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/pl_trace_$TAG.txt
for cfg in ${RUNS:-"c3:" "c2:--workload c2"}; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_$name.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$name', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'])"
done
