# Cout = 192 igemm: 256 x 192 whole-width tiles (ITTS_IG192=1, default) vs 256 x 64 tiles (0)
set -o pipefail
for v in 1 0; do
  echo "ITTS_IG192=$v"
  ITTS_IG192=$v timeout -k 10 150 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward|'conv'" || exit 1
done
