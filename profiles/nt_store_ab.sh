# non-temporal output stores (ubench_libs/libitts_nt.so, -DITTS_NT_STORE=1) vs the default build:
# C3 bench, interleaved runs
set -o pipefail
for lib in default nt default nt; do
  if [ "$lib" = default ]; then unset ITTS_HIP_LIB; else export ITTS_HIP_LIB=$PWD/ubench_libs/libitts_$lib.so; fi
  timeout -k 10 300 python3 bench.py --no-cpu-baseline > /tmp/b_$lib.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('/tmp/b_$lib.json').read().strip().splitlines()[-1]);print('lib=$lib', d['value'], 'audio-s/s', d['ms_per_step'], 'ms/batch, decode step', d['roofline']['avg_launch_us'], 'us, act', d['roofline_vocoder_act']['frac'], 'amp', d['roofline_vocoder_amp']['frac'], 'conv', d['roofline_vocoder_conv']['frac'])"
done
