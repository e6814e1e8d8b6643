# igemm tile-config build variants (ITTS_HIPCC_DEFS builds in ubench_libs/): vocoder forward time and
# per-launch us of the igemm convs (C >= 192) from profiles/ubench_vocoder.py
set -o pipefail
for lib in ${LIBS:-default}; do
  echo "lib=$lib"
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$lib; fi
  timeout -k 10 120 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward|'conv'" || exit 1
done
