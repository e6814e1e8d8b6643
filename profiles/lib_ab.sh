# decode step time (us, HIP events per graph replay) and C3 throughput per library build variant
set -o pipefail
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$lib; fi
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$lib', d['roofline']['avg_launch_us'], d['value'])"
done
