#!/bin/bash
# Time microbench shapes with the in-tree library and with variant builds under build/var/.
# usage: tools/variant_run.sh "<shape-substr list>" "<cfgs>"
set -e
for v in base build/var/lib_*.so; do
  if [ $v = base ]; then unset SMPQ_LIB; else export SMPQ_LIB=$v; fi
  echo "== $v"
  for s in $1; do timeout -k 10 100 python3 tools/conv_microbench.py 3 static $s $2 2>&1 | grep -v amdgpu; done
done
