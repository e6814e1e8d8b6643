#!/bin/bash
# decode-step tail (mel_head fold_last, sample_embed prefetch): tests, kernel microbenchmark, C3 / C2 bench lines
set -o pipefail
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_decode_tail.py tests/test_gpu_abi_decode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tail_tests_$tag.txt 2>&1 || { tail -40 gpurun_out/tail_tests_$tag.txt; exit 1; }
tail -1 gpurun_out/tail_tests_$tag.txt
timeout -k 10 200 python3 profiles/ubench_tail.py 2>&1 | grep -v amdgpu.ids || exit 1
for lib in new old; do
  if [ $lib = old ]; then export ITTS_HIP_LIB=index-tts-dubbing_amd/indextts/libitts_hip_ab.so; fi
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > gpurun_out/bench_${tag}_c3_$lib.json 2>/dev/null || exit 1
  timeout -k 10 300 python3 -u bench.py --workload c2 --no-cpu-baseline > gpurun_out/bench_${tag}_c2_$lib.json 2>/dev/null || exit 1
  for w in c3 c2; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), d.get('ms_per_step'))" gpurun_out/bench_${tag}_${w}_$lib.json "$w $lib"; done
done
