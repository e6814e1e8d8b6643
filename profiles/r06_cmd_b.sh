set -o pipefail
mkdir -p gpurun_out
export ITTS_PARITY_TAG=r06b
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_pl.py tests/test_gpu_vocoder.py tests/test_gpu_parity_bf16.py -k "beams_equal_chain or bit_identical or fused_tail or vocoder or beam_search_sets" > gpurun_out/tests_r06b.txt 2>&1 || { echo tests failed; tail -40 gpurun_out/tests_r06b.txt; exit 1; }
tail -3 gpurun_out/tests_r06b.txt
bash profiles/r06_b3nt.sh r06b
