#!/bin/bash
# Round-6 profiling pass (run from the repo root via gpurun): rocprofv3 kernel stats of bench.py (C3 default
# path), the FETCH_SIZE / WRITE_SIZE passes of the decode step (greedy C3 on the persistent layers and on the launch
# chain, beam3 on the persistent layers: beam-major attention) and of the vocoder
#   -> gpurun_out/{kernel_stats_$TAG.{csv,txt}, traffic_decode_{pl,chain,beam3}_$TAG.json, traffic_vocoder_$TAG.json}
set -e
export TMPDIR=/tmp
TAG=${1:-r06}
mkdir -p gpurun_out
rm -rf /tmp/prof /tmp/pmc_*
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof_$TAG.log 2>&1
cp "$(find /tmp/prof -name '*kernel_stats.csv' | head -n 1)" gpurun_out/kernel_stats_$TAG.csv
python3 profiles/summarize.py gpurun_out/kernel_stats_$TAG.csv 4 > gpurun_out/kernel_stats_$TAG.txt
echo stats-done
for run in pl chain beam3; do
  dec=$([ $run = beam3 ] && echo beam3 || echo greedy)
  plv=$([ $run = chain ] && echo 0 || echo 1)
  ITTS_PL=$plv timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_df_$run -o run -- python3 profiles/pmc_decode.py $dec > gpurun_out/pmc_df_$run.log 2>&1
  ITTS_PL=$plv timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc_dw_$run -o run -- python3 profiles/pmc_decode.py $dec > gpurun_out/pmc_dw_$run.log 2>&1
  python3 profiles/traffic.py decode /tmp/pmc_df_$run /tmp/pmc_dw_$run > gpurun_out/traffic_decode_${run}_$TAG.json
  echo $run-done
done
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pmc_vf -o run -- python3 profiles/pmc_vocoder.py > gpurun_out/pmc_vf.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/pmc_vw -o run -- python3 profiles/pmc_vocoder.py > gpurun_out/pmc_vw.log 2>&1
python3 profiles/traffic.py vocoder /tmp/pmc_vf /tmp/pmc_vw > gpurun_out/traffic_vocoder_$TAG.json
echo profiles-done
