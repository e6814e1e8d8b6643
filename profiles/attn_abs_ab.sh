# (round 3 experiment, removed after this A/B) decode attention with absolute key positions (ubench_libs/libitts_abs.so, -DITTS_ATTN_ABS=1: the first
# round's K/V addresses independent of the step counter and padding) vs the default: attention tests
# on the variant, then the C3 bench interleaved
set -o pipefail
ITTS_HIP_LIB=$PWD/ubench_libs/libitts_abs.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "attn_decode" 2>&1 | tail -2 || exit 1
for lib in default abs default abs; do
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$PWD/ubench_libs/libitts_$lib.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > /tmp/b_$lib.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('/tmp/b_$lib.json').read().strip().splitlines()[-1]);print('lib=$lib', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/batch, decode step', d['roofline']['avg_launch_us'], 'us')"
done
