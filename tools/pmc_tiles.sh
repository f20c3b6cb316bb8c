#!/bin/bash
# PMC screen of tile configs on one tools/tile_bench.py shape (separate --pmc passes, kernel trace
# only). usage: tools/pmc_tiles.sh <cfg,cfg,...> <shape-substr> <outdir>
export TMPDIR=/tmp
C=$1; S=$2; O=$3
mkdir -p $O
run() { timeout -k 10 120 rocprofv3 --pmc $1 --output-format csv -d $O/$2 -o run -- python3 tools/tile_bench.py $C $S > $O/$2.log 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" p1 && \
run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p2 && \
python3 tools/pmc_summary.py $O/p1 $O/p2 > $O/summary.txt
