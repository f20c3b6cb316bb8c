#!/bin/bash
# Memory-pipeline PMC counters (TA / TD / TCP / TCC), small separate passes, for one microbench shape.
# usage: tools/pmc_mem.sh <limbs> <shape-substr> <cfgs> <outdir>
export TMPDIR=/tmp
L=$1; S=$2; C=$3; O=$4
mkdir -p $O
run() { timeout -k 5 90 rocprofv3 --pmc $1 --output-format csv -d $O/$2 -o run -- python3 tools/conv_microbench.py $L static $S $C > $O/$2.log 2>&1; }
run "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" m1 && run "TA_ADDR_STALLED_BY_TC_CYCLES_sum" m2 && \
run "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum" m3 && run "TCP_PENDING_STALL_CYCLES_sum" m4 && \
run "TD_TD_BUSY_sum" m5 && run "TCC_BUSY_sum" m6 && \
run "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD" m7
