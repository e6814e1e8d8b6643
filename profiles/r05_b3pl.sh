# beam3 on the persistent layers: PL tests, beam3 bench chain (ITTS_PL_MAX_ROWS=32) vs PL (96), the 96-row trace
set -o pipefail
TAG=${1:-r05r}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_tests_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/pl_tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for mr in 32 96; do
  ITTS_PL_MAX_ROWS=$mr timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --decoding beam3 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('beam3 maxrows=$mr', d['roofline']['avg_launch_us'], d['value'])"
done
done
ITTS_PL_MAX_ROWS=128 ITTS_HIP_LIB=$PWD/index-tts-dubbing_amd/indextts/libitts_hip_trace.so STEPS=400 timeout -k 10 300 python3 profiles/pl_trace.py 96 > gpurun_out/pl_trace_${TAG}_96.txt 2>&1 && grep -v amdgpu gpurun_out/pl_trace_${TAG}_96.txt | head -24
