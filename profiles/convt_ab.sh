# ConvTranspose up-samplers: phases as output columns of ONE implicit GEMM (ITTS_VOC_CONVT_FUSED=1,
# default: stages with kernel == stride) vs one launch per phase (0); this A/B ran with the C <= 96 k = 2u stages fused too
set -o pipefail
for v in 1 0; do
  echo "ITTS_VOC_CONVT_FUSED=$v"
  ITTS_VOC_CONVT_FUSED=$v timeout -k 10 150 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward|'conv', (1536|768|384|192|96|48), (1|2|3)\)" || exit 1
done
