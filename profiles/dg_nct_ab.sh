# (round 3 experiment, removed after this A/B) beam decode: c_fc (96 rows, 320 column tiles) with two 16-column tiles per workgroup vs one
# (ITTS_DG_NCT=1): bit-identity tests, then the beam3 C3 bench interleaved
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "decode_gemm16x" 2>&1 | tail -2 || exit 1
for v in 2 1 2 1; do
  ITTS_DG_NCT=$v timeout -k 10 300 python3 bench.py --decoding beam3 --no-cpu-baseline --no-kernel-timing > /tmp/b_$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('/tmp/b_$v.json').read().strip().splitlines()[-1]);print('ITTS_DG_NCT=$v', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/batch')"
done
