# beam3 C3 bench A/B (round 3): the measured variants were a per-utterance beam attention kernel
# (ITTS_ATTN_BEAMS=1, since removed) and the per-row lineage kernel at 10 / 4 keys per round
# (ITTS_ATTN_ROWS_KB, since folded into the default: 4 for the lineage form).  Now: default vs
# ITTS_ATTN_SMALLKB=0 (10 keys per round everywhere).
set -o pipefail
mkdir -p gpurun_out
for v in 1 0; do
  ITTS_ATTN_SMALLKB=$v timeout -k 10 300 python3 bench.py --decoding beam3 --no-cpu-baseline --no-kernel-timing > gpurun_out/beam3_smallkb$v.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/beam3_smallkb$v.json').read().strip().splitlines()[-1]);print('ITTS_ATTN_SMALLKB=$v', d['value'], 'audio-s/s', d['ms_per_step'], 'ms per batch')"
done
