# vocoder per-launch timings across library builds (profiles/ubench_vocoder.py)
set -o pipefail
for lib in ${LIBS:-default}; do
  echo "lib=$lib"
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$lib; fi
  timeout -k 10 120 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "${PAT:-forward \(C|conv}" || exit 1
done
