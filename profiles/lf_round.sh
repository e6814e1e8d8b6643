# lane-reuse bug probes: the first-step debug dump, then the pass/fail probe per library variant
L=$PWD/index-tts-dubbing_amd/indextts
mkdir -p gpurun_out
ITTS_HIP_LIB=$L/libitts_hip_dbg.so timeout -k 10 300 python -u profiles/lf_dbg.py > gpurun_out/lf_dbg.txt 2>&1 || exit 1
grep "call\|wg\|codes" gpurun_out/lf_dbg.txt | grep -v "^>>"
for v in default sys acq; do
  if [ $v = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$L/libitts_hip_$v.so; fi
  timeout -k 10 300 python -u profiles/lf_check.py > gpurun_out/lf_check_$v.txt 2>&1 || exit 1
  grep "^LIB" gpurun_out/lf_check_$v.txt
done
