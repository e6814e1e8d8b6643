#!/bin/bash
# single-owner phase D + side-by-side beam merges (product) vs HEAD before them (libitts_hip_ab.so): PL/ABI tests,
# then C3 greedy / beam3 / C2 bench lines interleaved, then phase traces (trace build) at 32 rows and beam3 96 rows.
# usage: bash profiles/r06_dow.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
AB=index-tts-dubbing_amd/indextts/libitts_hip_ab.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pl.py tests/test_gpu_abi_decode.py > gpurun_out/tests_$tag.txt 2>&1 || { echo tests failed; tail -30 gpurun_out/tests_$tag.txt; exit 1; }
tail -2 gpurun_out/tests_$tag.txt
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_${tag}_$name.json 2> gpurun_out/ab_${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/ab_${tag}_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), d.get('ms_per_step'))" gpurun_out/ab_${tag}_$name.json $name
}
C3="python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline"
B3="python -u bench.py --decoding beam3 --steps 3 --warmup 1 --no-cpu-baseline"
for rep in 1 2; do
  run c3_new_$rep $C3 && run c3_old_$rep ITTS_HIP_LIB=$AB $C3 && run b3_new_$rep $B3 && run b3_old_$rep ITTS_HIP_LIB=$AB $B3 || exit 1
done
run c2_new python -u bench.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline && run c2_old ITTS_HIP_LIB=$AB python -u bench.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline || exit 1
T=index-tts-dubbing_amd/indextts/libitts_hip_trace.so
STEPS=400 ITTS_HIP_LIB=$T timeout -k 10 300 python -u profiles/pl_trace.py 32 > gpurun_out/pl_trace_${tag}_32.txt 2>&1 && \
BEAMS=3 STEPS=400 ITTS_HIP_LIB=$T timeout -k 10 300 python -u profiles/pl_trace.py 96 > gpurun_out/pl_trace_${tag}_b96.txt 2>&1 || { echo trace failed; exit 1; }
grep -v amdgpu.ids gpurun_out/pl_trace_${tag}_32.txt gpurun_out/pl_trace_${tag}_b96.txt | grep "span\|E2 o\|D x1\|E4 x1\|B attention\|G end"
