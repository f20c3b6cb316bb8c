set -e
for a in base 1 2 8 16 34; do
  if [ $a = base ]; then export SMPQ_LIB=""; unset SMPQ_LIB; else export SMPQ_LIB=build/ablate/lib$a.so; fi
  echo "== ablate $a"
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c3_64_256 21,24,14 2>&1 | grep -v amdgpu
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c2_256_256 30,14 2>&1 | grep -v amdgpu
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static c1_256_64 9,23 2>&1 | grep -v amdgpu
done
