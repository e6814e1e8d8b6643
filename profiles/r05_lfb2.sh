# long-form chunk size, wider: srt_dubbing's decoding at 64 / 128 / 256 utterances per chunk (192 / 384 / 768 beam
# rows, launch chain), greedy at 128 (persistent layers) / 256 (chain), interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for cfg in "srt:64" "srt:128" "srt:256" "greedy:128" "greedy:256"; do
  dec=${cfg%%:*}; n=${cfg#*:}
  ITTS_LONGFORM_BATCH=$n timeout -k 10 300 python3 bench.py --workload c5 --c5-decoding $dec --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('c5 $dec chunk=$n', d['value'], d['ms_per_step'])"
done
done
