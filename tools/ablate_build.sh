#!/bin/bash
# Diagnostics: build libsmpq variants with compile-time ablations of the LDS-DMA conv kernel
# (-DSMPQ_DIAG_ABLATE=N, results are wrong) into ./abl/libN.so (in-tree so they travel to the GPU box).
# usage: tools/ablate_build.sh "1 2 4 8 16"
set -e
cd "$(dirname "$0")/.."
C=semilayer-wise-mixed-precision-quantization_amd/csrc
OUT=abl
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
for a in $1; do
  ( /opt/rocm/bin/hipcc $F -DSMPQ_DIAG_ABLATE=$a -c $C/conv_glds.hip -o $OUT/g$a.o 2>/dev/null ) &
done
for s in abi quant conv eval fingerprint; do ( /opt/rocm/bin/hipcc $F -c $C/$s.hip -o $OUT/$s.o 2>/dev/null ) & done
wait
for a in $1; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib$a.so $OUT/abi.o $OUT/quant.o $OUT/conv.o $OUT/eval.o $OUT/fingerprint.o $OUT/g$a.o
done
rm -f $OUT/*.o
