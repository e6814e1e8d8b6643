# last check of the in-tree build at HEAD: PL + ABI decode tests, smoke, the default bench line
set -o pipefail
TAG=${1:-r05last}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py tests/test_gpu_abi_decode.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || exit 1
tail -1 gpurun_out/smoke_$TAG.txt
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]);r=d['roofline'];print('c3', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'], d['cpu_baseline']['value'])"
