# lane-reuse stress: per-call cue loop passes with the persistent layers, product build vs memset-node build
L=$PWD/index-tts-dubbing_amd/indextts
mkdir -p gpurun_out
for v in ${VARIANTS:-memset default}; do
  if [ $v = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$L/libitts_hip_$v.so; fi
  timeout -k 10 400 python -u profiles/lf_stress.py > gpurun_out/lf_stress_$v.txt 2>&1 || exit 1
  grep "^LIB" gpurun_out/lf_stress_$v.txt
done
