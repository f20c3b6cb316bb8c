#!/bin/bash
# Two PMC passes (instruction mix / wave occupancy) for one microbench shape and tile set.
# usage: tools/pmc_quick.sh <limbs> <shape-substr> <cfgs> <outdir>
export TMPDIR=/tmp
L=$1; S=$2; C=$3; O=$4
mkdir -p $O
run() { timeout -k 10 240 rocprofv3 --pmc $1 --output-format csv -d $O/$2 -o run -- python3 tools/conv_microbench.py $L static $S $C > $O/$2.log 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" p1 && \
run "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM" p2
