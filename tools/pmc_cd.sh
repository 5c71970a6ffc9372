set -u
export TMPDIR=/tmp
MURR_DECODE_VERBOSE=1 timeout -k 10 120 python3 bench.py --config C --blocks 10 --steps 5 --warmup 2 --no-cpu > gpurun_out/C_bench.log 2>&1 || exit 1
MURR_DECODE_VERBOSE=1 timeout -k 10 120 python3 bench.py --config D --steps 10 --warmup 2 --no-cpu > gpurun_out/D1_bench.log 2>&1 || exit 1
OUT=gpurun_out/pmcC BENCH_ARGS="--config C --blocks 10 --steps 2 --warmup 1 --no-cpu" bash tools/pmc.sh || exit 1
OUT=gpurun_out/pmcB BENCH_ARGS="--steps 2 --warmup 1 --no-cpu" PMC_LIST="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM
SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_FLAT
TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT" bash tools/pmc.sh || exit 1
