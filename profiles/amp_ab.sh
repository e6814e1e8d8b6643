# amp_conv build variants (ITTS_HIPCC_DEFS builds in ubench_libs/) x vocoder AMP-layer modes:
# per-launch us of the amp / act kernels from profiles/ubench_vocoder.py
set -o pipefail
for lib in ${LIBS:-default}; do
  for f in ${MODES:-default}; do
    echo "lib=$lib ITTS_VOC_FUSED=$f"
    if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$lib; fi
    if [ "$f" = default ]; then unset ITTS_VOC_FUSED; elif [ "$f" = none ]; then export ITTS_VOC_FUSED=; else export ITTS_VOC_FUSED=$f; fi
    timeout -k 10 120 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward \(C|'amp'|'act', (24|48|96)" || exit 1
  done
done
