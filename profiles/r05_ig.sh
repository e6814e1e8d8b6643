# igemm256 tile variants on the latent-pass GEMMs (profiles/ubench_ig256.py), interleaved
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for v in ${VARIANTS:-3 4}; do
  echo "== variant $v"
  ITTS_IG256_VARIANT=$v timeout -k 10 120 python3 profiles/ubench_ig256.py 2>&1 | grep -v amdgpu.ids || exit 1
done
done
for args in "" "--workload c2"; do
  timeout -k 10 180 python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 $args > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]); print('bench $args', d['roofline']['avg_launch_us'], d['value'])"
done
