#!/bin/bash
# PMC counters (4 separate --pmc passes, kernel trace only) for one microbench shape / tile set.
# usage: tools/pmc_shape.sh <limbs> <shape-substr> <cfgs> <outdir>
export TMPDIR=/tmp
L=$1; S=$2; C=$3; O=$4
mkdir -p $O
run() { timeout -k 10 240 rocprofv3 --pmc $1 --output-format csv -d $O/$2 -o run -- python3 tools/conv_microbench.py $L static $S $C > $O/$2.log 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" p1 && \
run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p2 && \
run "FETCH_SIZE" p3 && run "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" p4
