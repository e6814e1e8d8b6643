set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pl.py tests/test_gpu_abi_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pl_tests_r05p.txt 2>&1
rc=$?; tail -2 gpurun_out/pl_tests_r05p.txt; [ $rc -eq 0 ] || exit $rc
LPLS="1 20" bash profiles/r05_lpl.sh r05p_ab 2>&1 | grep lpl
