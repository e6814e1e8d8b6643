# amp_conv build variants (ITTS_HIPCC_DEFS builds in ubench_libs/): vocoder per-launch timings
set -o pipefail
for lib in ${LIBS:-default ubench_libs/lib_late.so}; do
  echo "lib=$lib"
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$lib; fi
  timeout -k 10 120 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward \(C|'amp', (24|48)" || exit 1
done
