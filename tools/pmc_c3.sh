export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 tools/conv_microbench.py 3 static c3 1,7,12,13,14,15,16,17,18,19,20,21 > gpurun_out/mb.log 2>&1
Q="3 static c3_64_256_56 7,19,20"
run() { timeout -k 10 240 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/$2 -o run -- python3 tools/conv_microbench.py $3 $4 $5 $6 > gpurun_out/$2.log 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" p1 $Q && \
run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p2 $Q && \
run "FETCH_SIZE" p3 $Q && run "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" p4 $Q
