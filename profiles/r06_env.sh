#!/bin/bash
# env A/B (round 6): kernel arguments in device memory (HIP_FORCE_DEV_KERNARG) for C3 / C2, and the srt_dubbing
# long-form decoding (C5, beam sample 3) in 32-utterance chunks (96 beam rows: persistent layers, beam-major) vs
# 128-utterance chunks (384 rows: the launch chain).  usage: bash profiles/r06_env.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 400 env "$@" > gpurun_out/env_${tag}_$name.json 2> gpurun_out/env_${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/env_${tag}_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), d.get('ms_per_step'))" gpurun_out/env_${tag}_$name.json $name
}
C3="python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline"
C2="python -u bench.py --workload c2 --steps 4 --warmup 1 --no-cpu-baseline"
for rep in 1 2; do
  run c3_kdef_$rep $C3 && run c3_kdev_$rep HIP_FORCE_DEV_KERNARG=1 $C3 && run c3_khost_$rep HIP_FORCE_DEV_KERNARG=0 $C3 || exit 1
done
run c2_kdef $C2 && run c2_kdev HIP_FORCE_DEV_KERNARG=1 $C2 && run c2_khost HIP_FORCE_DEV_KERNARG=0 $C2 || exit 1
C5="python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing"
run c5_lf128 $C5 && run c5_lf32 ITTS_LONGFORM_BATCH=32 $C5 && run c5_lf96 ITTS_LONGFORM_BATCH=96 $C5
