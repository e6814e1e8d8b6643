# igemm WIDE tile-config build variants: latent-pass GEMM timings (profiles/ubench_latent.py) and the
# vocoder's non-window wide convs (ConvTranspose phases)
set -o pipefail
for lib in ${LIBS:-default}; do
  echo "lib=$lib"
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$lib; fi
  timeout -k 10 120 python3 profiles/ubench_latent.py 2>&1 | grep -E "wall|_gemm" || exit 1
  timeout -k 10 120 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "C call|'conv', (1536|768|384|1024), (1|2|7)\)" || exit 1
done
