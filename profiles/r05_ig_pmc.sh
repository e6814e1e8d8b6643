# PMC counters of the igemm256 latent-pass GEMMs (variant 3): wave-state split, LDS and MFMA activity
set -o pipefail
mkdir -p gpurun_out/igpmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 60 rocprofv3 -L > gpurun_out/igpmc/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" gpurun_out/igpmc/counters.txt | sort -u > gpurun_out/igpmc/sq_names.txt || true
wc -l gpurun_out/igpmc/sq_names.txt
REPS=3 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES -d gpurun_out/igpmc/p1 -o p1 --output-format csv -- python3 profiles/ubench_ig256.py > gpurun_out/igpmc/p1.log 2>&1
echo "p1 rc=$?"
