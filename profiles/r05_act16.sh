# (measured with ITTS_ACT_ST16 on by default; it is off by default since)
# activation kernel's 16-B output stores (ITTS_ACT_ST16=1, default) vs 8-B stores: vocoder tests (incl. the bit-
# identity of the two store forms), vocoder time at the C3 shape interleaved; synthesize_many's serial mode
# (pipeline tests + C3 --pipeline, whose 32-row batches now run back to back on the persistent layers)
set -o pipefail
TAG=${1:-r05ac}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_vocoder.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread -k "activation or synthesize or vocoder_c_forward or stage_local" > gpurun_out/voc_tests_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/voc_tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_pl.py -x -q --timeout 300 --timeout-method thread -k synthesize_many > gpurun_out/pl_many_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/pl_many_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for v in 1 0; do
  ITTS_ACT_ST16=$v timeout -k 10 120 python3 profiles/voc_time.py st16=$v 2>/dev/null || exit 1
done
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 --pipeline > gpurun_out/bench_${TAG}_c3pipe.json 2> gpurun_out/bench_${TAG}_c3pipe.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_c3pipe.json').read().strip().splitlines()[-1]); print('c3 pipeline', d['roofline']['avg_launch_us'], d['value'])"
timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench_${TAG}_c3.json').read().strip().splitlines()[-1]); print('c3 serial', d['roofline']['avg_launch_us'], d['value'], d['roofline_vocoder_act']['frac'], d['roofline_vocoder_act']['avg_launch_us'])"
