set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/r03s_bench_c3.json 2> gpurun_out/r03s_bench_c3.err || exit 1
tail -c 600 gpurun_out/r03s_bench_c3.json
rm -rf /tmp/prof2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof2 -o run -- python3 bench.py --workload c2 --no-cpu-baseline --no-kernel-timing > gpurun_out/r03s_c2_prof.log 2>&1 || exit 1
cp "$(find /tmp/prof2 -name '*kernel_stats.csv' | head -n 1)" gpurun_out/kernel_stats_c2_r03s.csv
python3 profiles/summarize.py gpurun_out/kernel_stats_c2_r03s.csv 3 > gpurun_out/kernel_stats_c2_r03s.txt
head -30 gpurun_out/kernel_stats_c2_r03s.txt
