# one-row steps with split softmax groups (SG): PL tests (PL == chain at B = 1 and 32), C2 / C3 decode steps with
# ITTS_PL_SPLITG=0 vs 1, interleaved
set -o pipefail
TAG=${1:-r05w}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py tests/test_gpu_abi_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_tests_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/pl_tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for sg in 0 1; do
  ITTS_PL_SPLITG=$sg timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --workload c2 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('c2 splitg=$sg', d['roofline']['avg_launch_us'], d['value'])"
done
done
for sg in 0 1; do
  ITTS_PL_SPLITG=$sg ITTS_HIP_LIB=$PWD/index-tts-dubbing_amd/indextts/libitts_hip_trace.so STEPS=400 timeout -k 10 300 python3 profiles/pl_trace.py 1 > gpurun_out/pl_trace_${TAG}_sg$sg.txt 2>&1 && echo "== sg=$sg" && grep -v amdgpu gpurun_out/pl_trace_${TAG}_sg$sg.txt | head -24
done
