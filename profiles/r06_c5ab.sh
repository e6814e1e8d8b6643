#!/bin/bash
# chain GEMM A/B (product vs ITTS_HIP_LIB=libitts_hip_ab.so): PL / ABI tests (PL = chain bit-identity), the
# long-form tests, then C5 srt_dubbing decoding and the beam3 chain (ITTS_PL=0) lines.  usage: bash profiles/r06_c5ab.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
AB=index-tts-dubbing_amd/indextts/libitts_hip_ab.so
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread tests/test_gpu_pl.py tests/test_gpu_abi_decode.py tests/test_gpu_longform.py tests/test_gpu_beam.py > gpurun_out/tests_$tag.txt 2>&1 || { echo tests failed; tail -30 gpurun_out/tests_$tag.txt; exit 1; }
tail -2 gpurun_out/tests_$tag.txt
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > gpurun_out/ab_${tag}_$name.json 2> gpurun_out/ab_${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/ab_${tag}_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), d.get('ms_per_step'))" gpurun_out/ab_${tag}_$name.json $name
}
C5="python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing"
B3C="python -u bench.py --decoding beam3 --steps 3 --warmup 1 --no-cpu-baseline"
run c5_new $C5 && run c5_old ITTS_HIP_LIB=$AB $C5 && run b3c_new ITTS_PL=0 $B3C && run b3c_old ITTS_PL=0 ITTS_HIP_LIB=$AB $B3C && \
run c5_new2 $C5 && run c5_old2 ITTS_HIP_LIB=$AB $C5
