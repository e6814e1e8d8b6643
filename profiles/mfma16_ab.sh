# igemm256 with 16x16x32 MFMA blocks (ubench_libs/libitts_m16.so, -DITTS_IG_MFMA16=1; the default since) vs the then-default
# 32x32x16: igemm tests on the variant, then vocoder convs and latent-pass GEMMs per launch
set -o pipefail
ITTS_HIP_LIB=$PWD/ubench_libs/libitts_m16.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_vocoder.py -k "igemm or convtranspose or vocoder_matches or ragged" 2>&1 | tail -2 || exit 1
for lib in default m16; do
  echo "== lib=$lib"
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$PWD/ubench_libs/libitts_$lib.so; fi
  timeout -k 10 150 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward|'conv', (768|384|192), (3|7|11)" || exit 1
  timeout -k 10 150 python3 profiles/ubench_latent.py 2>&1 | grep -E "wall|_gemm" || exit 1
done
