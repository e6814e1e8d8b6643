# vocoder AMP-layer modes per channel count: ITTS_VOC_FUSED lists the channel counts whose activation
# is fused into itts_amp_conv_fwd, ITTS_VOC_SPLIT those run as activation kernel + conv-only
# amp_conv; any other channel count runs activation kernel + igemm.  "-" = variable unset.
set -o pipefail
for m in ${MODES:-"-:-" "24,48:-" "-:24,48"}; do
  f=${m%%:*}; sp=${m#*:}
  echo "ITTS_VOC_FUSED=$f ITTS_VOC_SPLIT=$sp"
  if [ "$f" = - ]; then unset ITTS_VOC_FUSED; else export ITTS_VOC_FUSED=$f; fi
  if [ "$sp" = - ]; then unset ITTS_VOC_SPLIT; else export ITTS_VOC_SPLIT=$sp; fi
  timeout -k 10 120 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward|, (24|48|96), " || exit 1
done
