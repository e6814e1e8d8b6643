# one GPU pass over the persistent-layer work: PL bit-identity tests, phase traces of the trace builds,
# and PL / chain bench lines (C3); attn.c_proj epilogue A/B on the chain
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
L=$PWD/index-tts-dubbing_amd/indextts
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_test_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/pl_test_$TAG.txt; [ $rc -eq 0 ] || exit $rc
for v in ${TRACES:-trace}; do
  ITTS_HIP_LIB=$L/libitts_hip_$v.so timeout -k 10 200 python -u profiles/pl_trace.py 32 1 > gpurun_out/pl_${v}_$TAG.txt 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu.ids gpurun_out/pl_${v}_$TAG.txt
done
for cfg in ${RUNS:-"PL=1" "PL=0 OPROJ_EPI=0" "PL=0 OPROJ_EPI=1"}; do
  env $(echo $cfg | sed 's/\([A-Z_]*\)=/ITTS_\1=/g') timeout -k 10 300 python3 bench.py --no-cpu-baseline --steps 3 > gpurun_out/b.json 2> gpurun_out/b.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/b.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$cfg', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_us'])"
done
