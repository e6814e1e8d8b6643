#!/bin/bash
# Round-6 end pass on the current build: the whole GPU suite, smoke(), then the default bench line and the
# beam3 / C2 / C5 lines.  usage: bash profiles/r06_final.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out
export ITTS_PARITY_TAG=$tag
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/gpu_tests_$tag.txt 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_$tag.txt; exit 1; }
tail -2 gpurun_out/gpu_tests_$tag.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_$tag.txt; exit 1; }
tail -1 gpurun_out/smoke_$tag.txt
line() {
  local name=$1; shift
  timeout -k 10 400 "$@" > gpurun_out/bench_${tag}_$name.json 2> gpurun_out/bench_${tag}_$name.err || { echo "$name failed"; tail -5 gpurun_out/bench_${tag}_$name.err; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('avg_launch_us'), r.get('frac'), d.get('ms_per_step'))" gpurun_out/bench_${tag}_$name.json $name
}
line c3 python -u bench.py && line b3 python -u bench.py --decoding beam3 --no-cpu-baseline && \
line c2 python -u bench.py --workload c2 --no-cpu-baseline && \
line c5 python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing && \
line c5g python -u bench.py --workload c5 --c5-decoding greedy --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing
