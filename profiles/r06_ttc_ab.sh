#!/bin/bash
# conv-only AMP tile rows (ITTS_AMP_TTC*, never tuned apart from the fused-activation form): per-launch timings
set -o pipefail
for i in 1 2; do
  for lib in default "ubench_libs/lib_TTC96=256.so" "ubench_libs/lib_TTC32=512.so" "ubench_libs/lib_TTC64=128.so"; do
    echo "== $lib"
    if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$lib; fi
    timeout -k 10 120 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward \(C|'amp'" || exit 1
  done
done
