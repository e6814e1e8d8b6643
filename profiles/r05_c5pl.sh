# long-form chunks on the persistent layers: C5 greedy (128-row chunks) with ITTS_PL_MAX_ROWS=128 (every chunk on
# the persistent layers, so synthesize_many runs them back to back) vs the default 32 (chunks on the launch chain,
# decode of chunk i+1 overlapped with the back half of chunk i), interleaved; then the 128-row PL tests
set -o pipefail
TAG=${1:-r05c5}
mkdir -p gpurun_out
for rep in 1 2; do
for mr in 32 128; do
  ITTS_PL_MAX_ROWS=$mr timeout -k 10 300 python3 bench.py --workload c5 --c5-decoding greedy --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('c5 greedy maxrows=$mr', d['value'], d['ms_per_step'])"
done
done
