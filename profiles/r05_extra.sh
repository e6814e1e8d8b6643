# extra bench lines at HEAD: C5 long-form through IndexTTS.infer (srt_dubbing decoding and greedy), C3 --pipeline
set -o pipefail
TAG=${1:-r05z}
mkdir -p gpurun_out
for cfg in "c5srt:--workload c5 --c5-decoding srt --no-cpu-baseline" "c5greedy:--workload c5 --c5-decoding greedy --no-cpu-baseline" "c3pipe:--pipeline --no-cpu-baseline"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 python3 bench.py $args > gpurun_out/bench_${TAG}_$name.json 2> gpurun_out/bench_${TAG}_$name.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_$name.json').read().strip().splitlines()[-1]);print('$name', d['value'], d['ms_per_step'])"
done
