#!/bin/bash
# Round-2 ablation screen of the best tile per shape (tools/ablate_build.sh "4 8 12 16"):
# 4 no operand DMA, 8 no MFMA, 12 neither, 16 no epilogue. Diagnostics (results are wrong).
for a in base ${ABL:-4 8 12 16}; do
  if [ $a = base ]; then unset SMPQ_LIB; else export SMPQ_LIB=abl/lib$a.so; fi
  echo "== ablate $a"
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c2_256_256 42 2>&1 | grep -v amdgpu
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c2_64_64 15 2>&1 | grep -v amdgpu
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c1_1024_256 42 2>&1 | grep -v amdgpu
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c3_64_256 46 2>&1 | grep -v amdgpu
done
