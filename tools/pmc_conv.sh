export TMPDIR=/tmp
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
P="3 static c2_64_64_56 3,7"
Q="3 static c3_64_256_56 7,3"
run() { timeout -k 10 240 rocprofv3 --pmc $1 --output-format csv -d gpurun_out/$2 -o run -- python3 tools/conv_microbench.py $3 $4 $5 $6 > gpurun_out/$2.log 2>&1; }
run "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" p1a $P && \
run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p2a $P && \
run "FETCH_SIZE" p3a $P && run "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" p4a $P && \
run "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" p1b $Q && \
run "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" p2b $Q && \
run "FETCH_SIZE" p3b $Q && run "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum" p4b $Q
echo rc=$?
