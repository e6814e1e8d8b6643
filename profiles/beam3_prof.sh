# rocprofv3 kernel trace + stats of the beam3 C3 bench (the reference's default decoding)
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03}
mkdir -p gpurun_out
rm -rf /tmp/profb
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profb -o run -- \
    python3 bench.py --decoding beam3 --no-cpu-baseline --no-kernel-timing > gpurun_out/bench_prof_beam3_$TAG.log 2>&1 || exit 1
cp "$(find /tmp/profb -name '*kernel_stats.csv' | head -n 1)" gpurun_out/kernel_stats_beam3_$TAG.csv
python3 profiles/summarize.py gpurun_out/kernel_stats_beam3_$TAG.csv 3 > gpurun_out/kernel_stats_beam3_$TAG.txt
head -14 gpurun_out/kernel_stats_beam3_$TAG.txt
