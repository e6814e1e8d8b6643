# decode step per library variant (HIP events, bench.py 3 steps; C3, or ARGS="--workload c2" ...), interleaved;
# then (TRACE=1) the PL phase trace
set -o pipefail
TAG=${1:-r05b}
L=$PWD/index-tts-dubbing_amd/indextts
mkdir -p gpurun_out
for rep in 1 2; do
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$L/libitts_hip_$lib.so; fi
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 $ARGS > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$lib', d['roofline']['avg_launch_us'], d['value'])"
done
done
unset ITTS_HIP_LIB
if [ -n "$TRACE" ]; then
  for st in 40 400; do
    ITTS_HIP_LIB=$L/libitts_hip_trace.so STEPS=$st timeout -k 10 180 python3 profiles/pl_trace.py > gpurun_out/pl_trace_${TAG}_$st.txt 2>&1 || exit 1
    cat gpurun_out/pl_trace_${TAG}_$st.txt | grep -v amdgpu.ids
  done
fi
