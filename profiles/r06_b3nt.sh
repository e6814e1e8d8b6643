#!/bin/bash
# beam3 A/B (round 6): product = beam-major attention (one pass over an utterance's beams) + beam K/V loads with the
# default cache policy; rows = ITTS_PL_BEAM_SHARED=0 (row passes, default policy); old = row passes + non-temporal
# beam K/V loads (libitts_hip_ab.so built with -DITTS_BEAM_KV_NT=1).  Interleaved.  usage: bash profiles/r06_b3nt.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
AB=index-tts-dubbing_amd/indextts/libitts_hip_ab.so
run() {  # name, env..., args
  local name=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/b3ab_${tag}_$name.json 2> gpurun_out/b3ab_${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/b3ab_${tag}_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), d.get('ms_per_step'))" gpurun_out/b3ab_${tag}_$name.json $name
}
B3="python -u bench.py --decoding beam3 --steps 3 --warmup 1 --no-cpu-baseline --no-kernel-timing"
for rep in 1 2; do
  run b3_def_$rep $B3 && run b3_rows_$rep ITTS_PL_BEAM_SHARED=0 $B3 && run b3_old_$rep ITTS_HIP_LIB=$AB ITTS_PL_BEAM_SHARED=0 $B3 || exit 1
done
C5="python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing"
run c5_def $C5 && run c5_old ITTS_HIP_LIB=$AB ITTS_PL_BEAM_SHARED=0 $C5
