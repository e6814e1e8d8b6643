# end-of-round pass at HEAD: GPU suite + smoke + bench lines (profiles/r05_final.sh), then kernel stats and the
# PMC traffic passes (profiles/run_profiles_r05.sh: greedy C3 and beam3, both on the persistent layers now)
set -o pipefail
TAG=${1:-r05z}
bash profiles/r05_final.sh $TAG || exit $?
DECS="greedy beam3" bash profiles/run_profiles_r05.sh $TAG || exit $?
head -12 gpurun_out/kernel_stats_$TAG.txt
cat gpurun_out/traffic_decode_pl_$TAG.json gpurun_out/traffic_decode_beam3_$TAG.json
