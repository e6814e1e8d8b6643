#!/bin/bash
# mel_head GEMM with 16 waves per workgroup (ITTS_HIP_LIB=libitts_hip_ab.so, -DITTS_HEAD_NW=16) vs 8 (product):
# the full-size greedy parity tests on the 16-wave build, then C3 / C2 lines interleaved.  usage: bash profiles/r06_head.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
AB=index-tts-dubbing_amd/indextts/libitts_hip_ab.so
ITTS_HIP_LIB=$AB timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_fullsize.py tests/test_gpu_parity_bf16.py -k "c2 or c3 or greedy" > gpurun_out/tests_$tag.txt 2>&1 || { echo tests failed; tail -30 gpurun_out/tests_$tag.txt; exit 1; }
tail -2 gpurun_out/tests_$tag.txt
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/ab_${tag}_$name.json 2> gpurun_out/ab_${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/ab_${tag}_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), d.get('ms_per_step'))" gpurun_out/ab_${tag}_$name.json $name
}
C3="python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline"
C2="python -u bench.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline"
for rep in 1 2; do
  run c3_nw8_$rep $C3 && run c3_nw16_$rep ITTS_HIP_LIB=$AB $C3 || exit 1
done
run c2_nw8 $C2 && run c2_nw16 ITTS_HIP_LIB=$AB $C2
