# (round 3 experiment; the DMA form measured no faster and was removed)
# activation kernel: register-prefetch form (ITTS_ACT_DMA=0) vs LDS-DMA window form (1; 2 = 256-row
# jobs at C <= 32) at the vocoder's stage shapes, and resident-workgroup targets for the DMA form
set -o pipefail
for v in "0 768" "1 512" "1 768" "1 1024" "2 1024"; do
  set -- $v
  echo "== ITTS_ACT_DMA=$1 ITTS_ACT_DMA_WGS=$2"
  ITTS_ACT_DMA=$1 ITTS_ACT_DMA_WGS=$2 N=10 timeout -k 10 120 python3 profiles/ubench_act.py || exit 1
done
