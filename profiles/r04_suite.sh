# round-4 GPU pass: the GPU suite (measured parity values -> gpurun_out/parity_$TAG.json), smoke, the C3
# bench line (+ the RCCL gather at N = 1 via --dist), and an optional library A/B (LIBS="default x.so").
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
export ITTS_PARITY_TAG=$TAG
timeout -k 10 900 python -u -m pytest tests -m gpu -q ${PYTEST_X:-} --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$TAG.txt 2>&1
rc=$?
tail -4 gpurun_out/gpu_tests_$TAG.txt
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (numbers still recorded); anything else: stop
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || exit 1
tail -1 gpurun_out/smoke_$TAG.txt
timeout -k 10 300 python3 bench.py --breakdown > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err || exit 1
timeout -k 10 300 python3 bench.py --dist --no-cpu-baseline > gpurun_out/bench_${TAG}_c3_dist.json \
  2> gpurun_out/bench_${TAG}_c3_dist.err || exit 1
for f in c3 c3_dist; do
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_$f.json').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print('$f', d['value'], d['ms_per_step'], r.get('frac'), r.get('avg_launch_us'), d['config'].get('collective'))"
done
if [ -n "${LIBS:-}" ]; then bash profiles/lib_ab.sh; fi
