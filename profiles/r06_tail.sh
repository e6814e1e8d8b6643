set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_vocoder.py > gpurun_out/tests_r06t.txt 2>&1 || { echo tests failed; tail -30 gpurun_out/tests_r06t.txt; exit 1; }
tail -2 gpurun_out/tests_r06t.txt
timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/bench_r06t.json 2> gpurun_out/bench_r06t.err || { echo bench failed; tail -5 gpurun_out/bench_r06t.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_r06t.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['roofline_vocoder_tail'])"
