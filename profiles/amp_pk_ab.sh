# (round 3 experiment; the persistent form was removed after this measurement)
# persistent conv-only amp_conv (ITTS_AMP_PK=1, default) vs the one-tile form (0): per-launch us
set -o pipefail
for pk in 1 0; do
  echo "ITTS_AMP_PK=$pk"
  ITTS_AMP_PK=$pk timeout -k 10 150 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward|'amp'|'act'" || exit 1
done
