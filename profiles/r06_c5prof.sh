#!/bin/bash
# Kernel statistics of the C5 long-form workload (srt_dubbing's decoding: beam sample 3, 128-utterance chunks =
# 384 beam rows on the launch chain) -> gpurun_out/kernel_stats_c5_$TAG.{csv,txt}.  usage: bash profiles/r06_c5prof.sh TAG
set -e
export TMPDIR=/tmp
TAG=${1:-r06}
mkdir -p gpurun_out
rm -rf /tmp/prof_c5
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_c5 -o run -- \
    python3 bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-kernel-timing > gpurun_out/bench_c5prof_$TAG.log 2>&1
cp "$(find /tmp/prof_c5 -name '*kernel_stats.csv' | head -n 1)" gpurun_out/kernel_stats_c5_$TAG.csv
python3 profiles/summarize.py gpurun_out/kernel_stats_c5_$TAG.csv 2 > gpurun_out/kernel_stats_c5_$TAG.txt
head -30 gpurun_out/kernel_stats_c5_$TAG.txt
