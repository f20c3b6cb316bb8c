#!/bin/bash
# Texture-addresser / LDS / wave-state PMC screen of ONE conv launch shape (tools/bin/sb_time: the
# stamp bench without stamps, 128 ch x 64 px tile), one rocprofv3 --pmc pass per counter group.
#   usage (GPU box, repo root): bash tools/pmc_ta.sh "cin cout k hw bk" tag
set -e
export TMPDIR=/tmp
A=${1:-"256 256 3 14 64"}; T=${2:-c3x3_14_bk64}
O=gpurun_out/pmc_ta_$T
mkdir -p $O
i=0
for g in "TA_TA_BUSY TA_BUFFER_TOTAL_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
         "TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES GRBM_GUI_ACTIVE" \
         "TD_TD_BUSY TD_TC_STALL GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE" \
         "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  timeout -s KILL 60 rocprofv3 --pmc $g --output-format csv -d $O/p$i -o run -- ./tools/bin/sb_time $A > $O/p$i.log 2>&1
  i=$((i+1))
done
