#!/bin/bash
# Round-4 profiling pass (run from the repo root via gpurun): rocprofv3 kernel stats of bench.py (C3,
# persistent layers), and the FETCH_SIZE / WRITE_SIZE passes of the decode step for greedy and beam3 on
# the persistent layers (ITTS_PL=1) -> gpurun_out/{kernel_stats,traffic_decode*}_$TAG.*
set -e
export TMPDIR=/tmp
TAG=${1:-r04}
mkdir -p gpurun_out
rm -rf /tmp/prof /tmp/pmc_*
export ITTS_PL=${ITTS_PL:-1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof_$TAG.log 2>&1
cp "$(find /tmp/prof -name '*kernel_stats.csv' | head -n 1)" gpurun_out/kernel_stats_$TAG.csv
python3 profiles/summarize.py gpurun_out/kernel_stats_$TAG.csv 4 > gpurun_out/kernel_stats_$TAG.txt
sfx=$([ "$ITTS_PL" = 1 ] && echo _pl || echo "")
for dec in greedy beam3; do
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_df_$dec -o run -- python3 profiles/pmc_decode.py $dec > gpurun_out/pmc_df_$dec.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc_dw_$dec -o run -- python3 profiles/pmc_decode.py $dec > gpurun_out/pmc_dw_$dec.log 2>&1
  name=$([ $dec = greedy ] && echo traffic_decode${sfx} || echo traffic_decode_beam3${sfx})
  python3 profiles/traffic.py decode /tmp/pmc_df_$dec /tmp/pmc_dw_$dec > gpurun_out/${name}_$TAG.json
done
echo profiles-done
