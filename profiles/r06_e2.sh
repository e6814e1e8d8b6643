#!/bin/bash
# E2 as tagged granules (product) vs the counter hand-off (libitts_hip_ab.so = the previous commit): PL tests, then
# C3 greedy / C2 / beam3 bench lines interleaved.  usage: bash profiles/r06_e2.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
AB=index-tts-dubbing_amd/indextts/libitts_hip_ab.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pl.py tests/test_gpu_abi_decode.py > gpurun_out/tests_$tag.txt 2>&1 || { echo tests failed; tail -30 gpurun_out/tests_$tag.txt; exit 1; }
tail -2 gpurun_out/tests_$tag.txt
run() {
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/e2_${tag}_$name.json 2> gpurun_out/e2_${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/e2_${tag}_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), d.get('ms_per_step'))" gpurun_out/e2_${tag}_$name.json $name
}
C3="python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline"
for rep in 1 2; do
  run c3_gran_$rep $C3 && run c3_cnt_$rep ITTS_HIP_LIB=$AB $C3 || exit 1
done
run c2_gran python -u bench.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline && run c2_cnt ITTS_HIP_LIB=$AB python -u bench.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline
run b3_gran python -u bench.py --decoding beam3 --steps 3 --warmup 1 --no-cpu-baseline && run b3_cnt ITTS_HIP_LIB=$AB python -u bench.py --decoding beam3 --steps 3 --warmup 1 --no-cpu-baseline
