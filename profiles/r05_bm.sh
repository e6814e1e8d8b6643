# beam rows utterance-major with phase A's row tiles gathered in the same order (libitts_hip_bm1.so, built with
# -DITTS_PL_BEAM_MAJOR=1) vs the default row-strided order: PL tests on the bm1 build, then beam3 interleaved
set -o pipefail
TAG=${1:-r05bm}
LIBD=$PWD/index-tts-dubbing_amd/indextts
mkdir -p gpurun_out
ITTS_HIP_LIB=$LIBD/libitts_hip_bm1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_tests_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/pl_tests_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in bm0 bm1; do
  if [ $v = bm1 ]; then L=$LIBD/libitts_hip_bm1.so; else L=$LIBD/libitts_hip.so; fi
  ITTS_HIP_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 --decoding beam3 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('b3 $v', d['roofline']['avg_launch_us'], d['value'])"
done
done
