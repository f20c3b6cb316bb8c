set -e
for a in base 2 16; do
  if [ $a = base ]; then unset SMPQ_LIB; else export SMPQ_LIB=build/ablate/lib$a.so; fi
  echo "== ablate $a"
  timeout -k 10 100 python3 tools/conv_microbench.py 3 static ds_64_256 2>&1 | grep -v amdgpu | tr '|' '\n'
done
