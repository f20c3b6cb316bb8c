#!/bin/bash
# Time representative shapes on the base library and on each ./abl/libN.so ablation (tools/ablate_build.sh).
for a in base ${ABL:-1 2 4 8 16}; do
  if [ $a = base ]; then unset SMPQ_LIB; else export SMPQ_LIB=abl/lib$a.so; fi
  echo "== ablate $a"
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c3_64_256 21,33 2>&1 | grep -v amdgpu
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c2_256_256 30,14 2>&1 | grep -v amdgpu
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c1_256_64 21,15 2>&1 | grep -v amdgpu
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c1_1024_256 33,30 2>&1 | grep -v amdgpu
done
