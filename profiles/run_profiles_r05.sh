#!/bin/bash
# Round-5 profiling pass (run from the repo root via gpurun): rocprofv3 kernel stats of bench.py (C3 default
# path), the FETCH_SIZE / WRITE_SIZE passes of the decode step (greedy C3 on the persistent layers; beam3 on
# the launch chain) and of the vocoder
#   -> gpurun_out/{kernel_stats_$TAG.{csv,txt}, traffic_decode_pl_$TAG.json, traffic_decode_beam3_$TAG.json,
#                  traffic_vocoder_$TAG.json}
set -e
export TMPDIR=/tmp
TAG=${1:-r05}
mkdir -p gpurun_out
rm -rf /tmp/prof /tmp/pmc_*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof_$TAG.log 2>&1
cp "$(find /tmp/prof -name '*kernel_stats.csv' | head -n 1)" gpurun_out/kernel_stats_$TAG.csv
python3 profiles/summarize.py gpurun_out/kernel_stats_$TAG.csv 4 > gpurun_out/kernel_stats_$TAG.txt
for dec in ${DECS:-greedy beam3}; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_df_$dec -o run -- python3 profiles/pmc_decode.py $dec > gpurun_out/pmc_df_$dec.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc_dw_$dec -o run -- python3 profiles/pmc_decode.py $dec > gpurun_out/pmc_dw_$dec.log 2>&1
  name=$([ $dec = greedy ] && echo traffic_decode_pl || echo traffic_decode_beam3)
  python3 profiles/traffic.py decode /tmp/pmc_df_$dec /tmp/pmc_dw_$dec > gpurun_out/${name}_$TAG.json
done
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_vf -o run -- python3 profiles/pmc_vocoder.py > gpurun_out/pmc_vf.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc_vw -o run -- python3 profiles/pmc_vocoder.py > gpurun_out/pmc_vw.log 2>&1
python3 profiles/traffic.py vocoder /tmp/pmc_vf /tmp/pmc_vw > gpurun_out/traffic_vocoder_$TAG.json
echo profiles-done
