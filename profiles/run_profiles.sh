#!/bin/bash
# Profiling pass on the GPU box (run from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of bench.py (C3)  -> gpurun_out/kernel_stats.csv
#   2. FETCH_SIZE / WRITE_SIZE passes (one counter group per run) over the GPT decode step and the
#      vocoder                                            -> gpurun_out/traffic_{decode,vocoder}.json
# Large traces stay under /tmp on the box; only the small summaries come back.
set -e
export TMPDIR=/tmp
TAG=${1:-r02}
mkdir -p gpurun_out
rm -rf /tmp/prof /tmp/pmc_*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof_$TAG.log 2>&1
cp "$(find /tmp/prof -name '*kernel_stats.csv' | head -n 1)" gpurun_out/kernel_stats_$TAG.csv
# 4 batches under the profiler: warmup 1 + timed 2 + bench.py's instrumented vocoder step 1
python3 profiles/summarize.py gpurun_out/kernel_stats_$TAG.csv 4 > gpurun_out/kernel_stats_$TAG.txt
python3 profiles/copy_trace.py "$(find /tmp/prof -name '*kernel_trace.csv' | head -n 1)" > gpurun_out/copy_trace_$TAG.txt || true
if [ "${2:-pmc}" = "pmc" ]; then
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_df -o run -- python3 profiles/pmc_decode.py > gpurun_out/pmc_df.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc_dw -o run -- python3 profiles/pmc_decode.py > gpurun_out/pmc_dw.log 2>&1
  python3 profiles/traffic.py decode /tmp/pmc_df /tmp/pmc_dw > gpurun_out/traffic_decode_$TAG.json
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_vf -o run -- python3 profiles/pmc_vocoder.py > gpurun_out/pmc_vf.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc_vw -o run -- python3 profiles/pmc_vocoder.py > gpurun_out/pmc_vw.log 2>&1
  python3 profiles/traffic.py vocoder /tmp/pmc_vf /tmp/pmc_vw > gpurun_out/traffic_vocoder_$TAG.json
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_c -o run -- python3 profiles/pmc_calibrate.py > gpurun_out/pmc_c.log 2>&1
  python3 profiles/traffic.py calibrate /tmp/pmc_c > gpurun_out/traffic_calibration_$TAG.json
  # what bounds the vocoder's HBM-bound kernels: wave-state and instruction counters (two passes)
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv \
      -d /tmp/pmc_vsq -o run -- python3 profiles/pmc_vocoder.py > gpurun_out/pmc_vsq.log 2>&1
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --output-format csv \
      -d /tmp/pmc_vsi -o run -- python3 profiles/pmc_vocoder.py > gpurun_out/pmc_vsi.log 2>&1
  { python3 profiles/pmc_summary.py /tmp/pmc_vsq amp_conv aa_snake igemm;
    python3 profiles/pmc_summary.py /tmp/pmc_vsi amp_conv aa_snake igemm; } > gpurun_out/pmc_sq_vocoder_$TAG.txt
fi
echo profiles-done
