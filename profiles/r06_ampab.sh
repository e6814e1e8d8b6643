#!/bin/bash
# A/B of a vocoder kernel change: bit-identity of the vocoder PCM (product build vs ITTS_HIP_LIB=AB) and the
# per-launch timings of both builds.  usage: bash profiles/r06_ampab.sh TAG [AB_LIB]
set -o pipefail
tag=$1; ab=${2:-index-tts-dubbing_amd/indextts/libitts_hip_ab.so}
mkdir -p gpurun_out
timeout -k 10 120 python3 profiles/voc_dump.py gpurun_out/pcm_new_$tag.npy || exit 1
ITTS_HIP_LIB=$ab timeout -k 10 120 python3 profiles/voc_dump.py gpurun_out/pcm_old_$tag.npy || exit 1
python3 -c "import numpy as np,sys; a=np.load(sys.argv[1]); b=np.load(sys.argv[2]); print('pcm bit-identical:', a.shape==b.shape and bool((a==b).all()), int((a!=b).sum()))" gpurun_out/pcm_new_$tag.npy gpurun_out/pcm_old_$tag.npy
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_vocoder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/voc_tests_$tag.txt 2>&1 || { tail -30 gpurun_out/voc_tests_$tag.txt; exit 1; }
tail -1 gpurun_out/voc_tests_$tag.txt
for i in 1 2; do
  echo "== new"; timeout -k 10 200 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward \(C|'(amp|act)'" || exit 1
  echo "== old"; ITTS_HIP_LIB=$ab timeout -k 10 200 python3 profiles/ubench_vocoder.py 2>&1 | grep -E "forward \(C|'(amp|act)'" || exit 1
done
