# bench lines at HEAD: C3 greedy (the headline, with --breakdown), beam3, C5 (srt decoding, greedy), C2
set -o pipefail
TAG=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --breakdown > gpurun_out/bench_${TAG}_c3.json 2> gpurun_out/bench_${TAG}_c3.err || exit 1
tail -c 300 gpurun_out/bench_${TAG}_c3.json; grep -i "ms" gpurun_out/bench_${TAG}_c3.err | tail -12
timeout -k 10 300 python3 bench.py --decoding beam3 > gpurun_out/bench_${TAG}_c3_beam3.json 2>/dev/null || exit 1
timeout -k 10 400 python3 bench.py --workload c5 > gpurun_out/bench_${TAG}_c5_srt.json 2>/dev/null || exit 1
timeout -k 10 400 python3 bench.py --workload c5 --c5-decoding greedy > gpurun_out/bench_${TAG}_c5_greedy.json 2>/dev/null || exit 1
timeout -k 10 300 python3 bench.py --workload c2 > gpurun_out/bench_${TAG}_c2.json 2>/dev/null || exit 1
for f in c3 c3_beam3 c5_srt c5_greedy c2; do
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_$f.json').read().strip().splitlines()[-1]);r=d.get('roofline') or {};print('$f', d['value'], d['ms_per_step'], r.get('frac'), r.get('avg_launch_us'))"
done
