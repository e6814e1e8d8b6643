# the GPU test suite + smoke at HEAD (one process each, time-limited)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.txt 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_$TAG.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.txt 2>&1 || exit 1
cat gpurun_out/smoke_$TAG.txt | tail -1
