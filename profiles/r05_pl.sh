# round-5 persistent-layer hardening pass: PL / ABI tests, C3 + C2 bench lines, lane-reuse stress
set -o pipefail
TAG=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_pl.py tests/test_gpu_abi_decode.py -v --timeout 300 --timeout-method thread > gpurun_out/pl_tests_$TAG.txt 2>&1
rc=$?
tail -25 gpurun_out/pl_tests_$TAG.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for cfg in "c3:--breakdown" "c2:--workload c2 --no-cpu-baseline"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python3 bench.py $args > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_$name.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$name', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'])"
done
PASSES=6 timeout -k 10 300 python -u profiles/lf_stress.py > gpurun_out/lf_stress_$TAG.txt 2>&1 && grep "^LIB" gpurun_out/lf_stress_$TAG.txt
