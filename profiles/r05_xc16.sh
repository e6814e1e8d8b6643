# (measured with both switches ON in the default build; both are off by default since)
# A/B of two decode-layer switches, interleaved in one call:
#  * phase D x1^ copies as 16-B stores (ITTS_PL_XC16=1, default build) vs 4-B stores (libitts_hip_xc4.so, built with
#    ITTS_HIPCC_DEFS=-DITTS_PL_XC16=0): C3 and C2 decode steps
#  * beam lineage rows utterance-major (ITTS_PL_BEAM_MAJOR=1, default) vs row-strided (libitts_hip_bm0.so): beam3
# PL tests (default build) first.
set -o pipefail
TAG=${1:-r05xc}
LIBD=$PWD/index-tts-dubbing_amd/indextts
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py tests/test_gpu_abi_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_tests_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/pl_tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
run() {  # name lib bench-args...
  local name=$1 lib=$2; shift 2
  ITTS_HIP_LIB=$lib timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 "$@" > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('$name', d['roofline']['avg_launch_us'], d['value'])"
}
for rep in 1 2; do
  run "c3 xc16" $LIBD/libitts_hip.so --workload c3
  run "c3 xc4 " $LIBD/libitts_hip_xc4.so --workload c3
  run "c2 xc16" $LIBD/libitts_hip.so --workload c2
  run "c2 xc4 " $LIBD/libitts_hip_xc4.so --workload c2
  run "b3 bm1 " $LIBD/libitts_hip.so --decoding beam3
  run "b3 bm0 " $LIBD/libitts_hip_bm0.so --decoding beam3
done
