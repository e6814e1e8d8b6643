#!/bin/bash
# phase traces of the persistent layer (trace build) at the C3 greedy shape and beam3 (96 rows), then bench lines
# usage: bash profiles/r06_trace.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
T=index-tts-dubbing_amd/indextts/libitts_hip_trace.so
STEPS=400 ITTS_HIP_LIB=$T timeout -k 10 300 python -u profiles/pl_trace.py 32 > gpurun_out/pl_trace_${tag}_32.txt 2>&1 || { echo trace32 failed; tail gpurun_out/pl_trace_${tag}_32.txt; exit 1; }
BEAMS=3 STEPS=400 ITTS_HIP_LIB=$T timeout -k 10 300 python -u profiles/pl_trace.py 96 > gpurun_out/pl_trace_${tag}_b96.txt 2>&1 || { echo trace96 failed; tail gpurun_out/pl_trace_${tag}_b96.txt; exit 1; }
cat gpurun_out/pl_trace_${tag}_32.txt gpurun_out/pl_trace_${tag}_b96.txt | grep -v amdgpu.ids
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${tag}_c3.json 2> gpurun_out/bench_${tag}_c3.err || { echo bench c3 failed; exit 1; }
timeout -k 10 300 python -u bench.py --decoding beam3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_${tag}_b3.json 2> gpurun_out/bench_${tag}_b3.err || { echo bench b3 failed; exit 1; }
for f in c3 b3; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], d['value'], r['avg_launch_us'], r['frac'], d['ms_per_step'])" gpurun_out/bench_${tag}_$f.json $f; done
