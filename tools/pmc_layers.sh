#!/bin/bash
# Instruction mix and wave states of every quantized-conv launch of bench.py's eager roofline
# region (two rocprofv3 --pmc passes, kernel trace only), joined to the per-launch layer table by
# tools/pmc_layers.py. usage (GPU box, repo root): tools/pmc_layers.sh <outdir> [bench.py args, e.g.
# --config r34_4bit --batch 512]
export TMPDIR=/tmp
O=$1; shift; mkdir -p $O
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --layers $*"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 bench.py $ARGS > $O/p1.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 bench.py $ARGS > $O/p2.log 2>&1 && \
python3 tools/pmc_layers.py $O > $O/summary.txt
