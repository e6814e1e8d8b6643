#!/bin/bash
# A/B: beam K/V loads with the default cache policy (product) vs non-temporal (libitts_hip_ab.so built with
# -DITTS_BEAM_KV_NT=1), beam3 C3 and the C5 srt_dubbing decoding, interleaved.  usage: bash profiles/r06_b3nt.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
AB=index-tts-dubbing_amd/indextts/libitts_hip_ab.so
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/b3nt_${tag}_$name.json 2> gpurun_out/b3nt_${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/b3nt_${tag}_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), d.get('ms_per_step'))" gpurun_out/b3nt_${tag}_$name.json $name
}
for rep in 1 2; do
  run b3_def_$rep python -u bench.py --decoding beam3 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing && \
  run b3_nt_$rep ITTS_HIP_LIB=$AB python -u bench.py --decoding beam3 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing || exit 1
done
run c5_def python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing && \
run c5_nt ITTS_HIP_LIB=$AB python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing
