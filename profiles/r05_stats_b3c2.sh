# kernel stats of the beam3 and C2 bench lines (rocprofv3 --kernel-trace --stats)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in "b3:--decoding beam3" "c2:--workload c2"; do
  name=${w%%:*}; args=${w#*:}
  rm -rf /tmp/prof_$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o run -- \
      python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 $args > gpurun_out/bench_prof_$name.log 2>&1
  cp "$(find /tmp/prof_$name -name '*kernel_stats.csv' | head -n 1)" gpurun_out/kernel_stats_r05q_$name.csv
  python3 profiles/summarize.py gpurun_out/kernel_stats_r05q_$name.csv 3 > gpurun_out/kernel_stats_r05q_$name.txt
  head -16 gpurun_out/kernel_stats_r05q_$name.txt
done
