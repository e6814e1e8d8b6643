# (round 3 experiment, removed after this A/B) mel_head 257th column tile folded into workgroup 0 vs a 257th workgroup (ITTS_DG_EXTRA=0):
# bit-identity tests, then the C3 bench interleaved
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "decode_gemm" 2>&1 | tail -2 || exit 1
for v in 1 0 1 0; do
  ITTS_DG_EXTRA=$v timeout -k 10 300 python3 bench.py --no-cpu-baseline > /tmp/b_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('/tmp/b_$v.json').read().strip().splitlines()[-1]);print('ITTS_DG_EXTRA=$v', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/batch, decode step', d['roofline']['avg_launch_us'], 'us')"
done
