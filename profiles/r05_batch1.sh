# round-5 measurement batch 1: PL + vocoder GPU tests (gate), C2 small-step variants, C3 weight-policy variants,
# vocoder activation variants, beam3 line with the distinct-K/V accounting
set -o pipefail
TAG=${1:-r05e}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_pl.py tests/test_gpu_vocoder.py -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.txt 2>&1
rc=$?
tail -3 gpurun_out/tests_$TAG.txt
[ $rc -eq 0 ] || exit $rc
echo "== C2 (B = 1) per library"
LIBS="default kbs4 kbs8 kbs16 h32" ARGS="--workload c2" bash profiles/r05_ab.sh $TAG || exit 1
echo "== C3 weight cache policy"
VARIANTS="base ITTS_PL_KEEP_LAYERS=4 ITTS_PL_KEEP_LAYERS=8 ITTS_PL_KEEP_LAYERS=12" bash profiles/r05_env_ab.sh || exit 1
echo "== vocoder (ms) per library"
LIBS="default actS2 actS8 actW256 actW1024" bash profiles/voc_ab.sh || exit 1
ITTS_ACT_NB3=0 timeout -k 10 120 python3 profiles/voc_time.py nb3_off 2>/dev/null || exit 1
echo "== beam3"
timeout -k 10 300 python3 bench.py --decoding beam3 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/bench_${TAG}_b3.json 2> gpurun_out/bench_${TAG}_b3.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/bench_${TAG}_b3.json').read().strip().splitlines()[-1]);r=d['roofline'];print('b3', d['value'], r['avg_launch_us'], r['frac'], r['algorithmic_bytes_per_launch'])"
