# persistent layers vs the launch chain per row count (profiles/ubench_pl_rows.py), then the long-form / pipeline /
# lookahead GPU tests with every chunk of up to 128 rows on the persistent layers (ITTS_PL_MAX_ROWS=128)
set -o pipefail
TAG=${1:-r05rows}
mkdir -p gpurun_out
timeout -k 10 400 python3 -u profiles/ubench_pl_rows.py 32 64 96 128 2>&1 | grep -v amdgpu.ids | tee gpurun_out/pl_rows_$TAG.txt
[ ${PIPESTATUS[0]} -eq 0 ] || exit 1
ITTS_PL_MAX_ROWS=128 timeout -k 10 600 python -u -m pytest tests/test_gpu_longform.py tests/test_gpu_pipeline.py tests/test_gpu_lookahead.py tests/test_gpu_pl.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_rows128_$TAG.txt 2>&1
rc=$?; tail -2 gpurun_out/tests_rows128_$TAG.txt; exit $rc
