# vocoder AMP-layer modes with the MFMA activation kernel: fused act+conv (mode 1) vs activation
# kernel + conv-only kernel (mode 2) per channel count (ITTS_VOC_FUSED lists the fused ones)
set -o pipefail
for f in "24,48" "24" "48" ""; do
  echo "ITTS_VOC_FUSED=$f"
  ITTS_VOC_FUSED=$f timeout -k 10 120 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward \(C|'amp'|'act'" || exit 1
done
