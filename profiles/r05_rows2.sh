# PL_MAX_ROWS = 128 by default: the long-form / pipeline / lookahead / PL GPU tests, then C5 greedy and srt, C3
set -o pipefail
TAG=${1:-r05rows2}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_longform.py tests/test_gpu_pipeline.py tests/test_gpu_lookahead.py tests/test_gpu_pl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for cfg in "c5greedy:--workload c5 --c5-decoding greedy --no-cpu-baseline" "c5srt:--workload c5 --c5-decoding srt --no-cpu-baseline" "c3:--no-cpu-baseline"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python3 bench.py $args > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_$name.json').read().strip().splitlines()[-1]);print('$name', d['value'], d['ms_per_step'])"
done
