# long-form chunk size for srt_dubbing's decoding (beam sample 3): 128 utterances (384 beam rows: launch chain,
# decode overlapped with the back half) vs 42 (126 rows: persistent layers, batches back to back), interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for n in 128 42; do
  ITTS_LONGFORM_BATCH=$n timeout -k 10 300 python3 bench.py --workload c5 --c5-decoding srt --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('c5 srt chunk=$n', d['value'], d['ms_per_step'])"
done
done
