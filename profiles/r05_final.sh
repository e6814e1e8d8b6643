# round-5 GPU pass at HEAD: GPU suite (parity record), smoke, bench lines C3 (+breakdown) / C3 --dist / C2 / beam3,
# lane-reuse stress
set -o pipefail
TAG=${1:-r05}
mkdir -p gpurun_out
export ITTS_PARITY_TAG=$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.txt 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests_$TAG.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || exit 1
tail -1 gpurun_out/smoke_$TAG.txt
for cfg in "c3:--breakdown" "c3_dist:--dist --no-cpu-baseline" "c2:--workload c2 --no-cpu-baseline" "b3:--decoding beam3 --no-cpu-baseline"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python3 bench.py $args > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_$name.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$name', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'])"
done
grep breakdown gpurun_out/bench_${TAG}_c3.err
PASSES=6 timeout -k 10 300 python -u profiles/lf_stress.py > gpurun_out/lf_stress_$TAG.txt 2>&1 && grep "^LIB" gpurun_out/lf_stress_$TAG.txt
