# C3 decode step per library variant (HIP events), twice each, interleaved
set -o pipefail
L=$PWD/index-tts-dubbing_amd/indextts
for rep in 1 2; do
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$L/libitts_hip_$lib.so; fi
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$lib', d['roofline']['avg_launch_us'], d['value'])"
done
done
