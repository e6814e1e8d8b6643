set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python3 profiles/ubench_act.py > gpurun_out/act_mfma.txt 2>&1 && \
ITTS_ACT_MFMA=0 timeout -k 10 120 python3 profiles/ubench_act.py > gpurun_out/act_valu.txt 2>&1 && \
N=3 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d /tmp/pa1 -o run -- python3 profiles/ubench_act.py 96 > gpurun_out/pa1.log 2>&1 && \
N=3 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT --output-format csv -d /tmp/pa2 -o run -- python3 profiles/ubench_act.py 96 > gpurun_out/pa2.log 2>&1 && \
{ python3 profiles/pmc_summary.py /tmp/pa1 aa_snake; python3 profiles/pmc_summary.py /tmp/pa2 aa_snake; } > gpurun_out/pmc_act.txt
cat gpurun_out/act_mfma.txt gpurun_out/act_valu.txt gpurun_out/pmc_act.txt
