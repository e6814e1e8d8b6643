# MFMA activation kernel A/B across library builds (profiles/ubench_act.py, all stage shapes)
set -o pipefail
for lib in ${LIBS:-default}; do
  echo "lib=$lib"
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$lib; fi
  timeout -k 10 120 python3 profiles/ubench_act.py 2>&1 | grep "^act" || exit 1
done
