#!/bin/bash
# Diagnostics: build libsmpq variants with compile-time ablations of the LDS-DMA conv kernel and
# time one shape with each (results are wrong in ablated builds). usage: tools/ablate_glds.sh shape cfgs
set -e
cd "$(dirname "$0")/.."
C=semilayer-wise-mixed-precision-quantization_amd/csrc
OUT=${TMPDIR:-/tmp}/smpq_ablate
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
for a in ${ABL:-1 2 3 4 8}; do
  ( hipcc $F -DSMPQ_DIAG_ABLATE=$a -c $C/conv_glds.hip -o $OUT/g$a.o 2>/dev/null ) &
done
for s in abi quant conv; do ( hipcc $F -c $C/$s.hip -o $OUT/$s.o 2>/dev/null ) & done
wait
for a in ${ABL:-1 2 3 4 8}; do
  hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib$a.so $OUT/abi.o $OUT/quant.o $OUT/conv.o $OUT/g$a.o
done
echo "base"; python3 tools/conv_microbench.py 3 static "$1" "$2" 2>&1 | grep -v amdgpu
for a in ${ABL:-1 2 3 4 8}; do
  echo "ablate $a"; SMPQ_LIB=$OUT/lib$a.so python3 tools/conv_microbench.py 3 static "$1" "$2" 2>&1 | grep -v amdgpu
done
