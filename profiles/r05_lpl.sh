# multi-layer persistent launch: PL tests, then the decode step with ITTS_PL_LPL=1 (one launch per layer) vs the
# default (the whole step in one launch), C3 and C2, interleaved; then the phase trace of both (TRACE=1)
set -o pipefail
TAG=${1:-r05l}
L=$PWD/index-tts-dubbing_amd/indextts
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py tests/test_gpu_abi_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_tests_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/pl_tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for args in "" "--workload c2"; do
for rep in 1 2; do
for lpl in ${LPLS:-1 32}; do
  ITTS_PL_LPL=$lpl timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 $args > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$args lpl=$lpl', d['roofline']['avg_launch_us'], d['value'])"
done
done
done
if [ -n "$TRACE" ]; then
  for lpl in ${LPLS:-1 32}; do
    ITTS_PL_LPL=$lpl ITTS_HIP_LIB=$L/libitts_hip_trace.so STEPS=400 timeout -k 10 180 python3 profiles/pl_trace.py > gpurun_out/pl_trace_${TAG}_lpl$lpl.txt 2>&1 || exit 1
    echo "== lpl=$lpl"; grep -v amdgpu.ids gpurun_out/pl_trace_${TAG}_lpl$lpl.txt | head -30
  done
fi
