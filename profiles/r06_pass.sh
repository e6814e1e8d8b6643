#!/bin/bash
# Round-6 GPU pass: persistent-layer / ABI tests, vocoder tests, the bf16 parity tests, then a C3 bench line.
# usage: bash profiles/r06_pass.sh TAG [pytest files...]
set -o pipefail
tag=$1; shift
files=${@:-"tests/test_gpu_pl.py tests/test_gpu_abi_decode.py tests/test_gpu_vocoder.py tests/test_gpu_parity_bf16.py"}
mkdir -p gpurun_out
export ITTS_PARITY_TAG=$tag
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread $files > gpurun_out/tests_$tag.txt 2>&1 || { echo "tests failed rc=$?"; tail -30 gpurun_out/tests_$tag.txt; exit 1; }
tail -3 gpurun_out/tests_$tag.txt
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || { echo "bench failed"; tail -20 gpurun_out/bench_$tag.err; exit 1; }
cat gpurun_out/bench_$tag.json
