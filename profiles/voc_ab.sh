# vocoder time per library variant (profiles/voc_time.py), interleaved twice: LIBS="default actS2 ..."
set -o pipefail
L=$PWD/index-tts-dubbing_amd/indextts
for rep in 1 2; do
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$L/libitts_hip_$lib.so; fi
  timeout -k 10 120 python3 profiles/voc_time.py $lib 2>/dev/null || exit 1
done
done
