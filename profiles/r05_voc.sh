# round-5 vocoder pass: fused conv1 -> act2 tests, vocoder GPU tests, C3 bench with the phase breakdown (EPI on / off)
set -o pipefail
TAG=${1:-r05c}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_vocoder.py -v --timeout 300 --timeout-method thread -k "epilogue" > gpurun_out/voc_tests_$TAG.txt 2>&1
rc=$?
tail -8 gpurun_out/voc_tests_$TAG.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_vocoder.py -q --timeout 300 --timeout-method thread >> gpurun_out/voc_tests_$TAG.txt 2>&1
rc=$?
tail -3 gpurun_out/voc_tests_$TAG.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for rep in 1 2; do
for epi in "24,48" ""; do
  ITTS_VOC_EPI=$epi timeout -k 10 300 python3 bench.py --breakdown --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_${TAG}_epi.json 2> gpurun_out/bench_${TAG}_epi.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_epi.json').read().strip().splitlines()[-1]);print('epi=$epi', d['value'], d['ms_per_step'])"
  grep "breakdown" gpurun_out/bench_${TAG}_epi.err
done
done
