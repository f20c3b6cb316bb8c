#!/bin/bash
# Diagnostics: build libsmpq variants with compile-time ablations of the LDS-DMA conv kernel
# (-DSMPQ_DIAG_ABLATE=N, results are wrong) into ./abl/libN.so (in-tree so they travel to the GPU box).
# usage: tools/ablate_build.sh "1 2 4 8 16"   (STEM=1: ablate the fused stem, -DSMPQ_SP_DIAG=N, instead)
set -e
cd "$(dirname "$0")/.."
C=semilayer-wise-mixed-precision-quantization_amd/csrc
OUT=abl
mkdir -p $OUT
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off"
FAM="1,1 2,1 3,1 1,2 2,2 3,2 3,3"
if [ "${STEM:-0}" = 1 ]; then DEF=SMPQ_SP_DIAG; ABL="stem_pool"; FIXED="abi quant conv eval fingerprint conv_glds"
else DEF=SMPQ_DIAG_ABLATE; ABL="conv_glds"; FIXED="abi quant conv eval fingerprint stem_pool"; fi
for a in $1; do
  ( /opt/rocm/bin/hipcc $F -D$DEF=$a -c $C/$ABL.hip -o $OUT/g$a.o 2>/dev/null ) &
  for lw in $FAM; do  # the kernel's (L, LW) families (conv_glds_inst.hip)
    l=${lw%,*}; w=${lw#*,}
    if [ "${STEM:-0}" = 1 ]; then X=""; else X="-D$DEF=$a"; fi
    ( /opt/rocm/bin/hipcc $F $X -DSMPQ_INST_L=$l -DSMPQ_INST_LW=$w -c $C/conv_glds_inst.hip -o $OUT/i${a}_$l$w.o 2>/dev/null ) &
  done
  wait
done
for s in $FIXED; do ( /opt/rocm/bin/hipcc $F -c $C/$s.hip -o $OUT/$s.o 2>/dev/null ) & done
wait
for a in $1; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/lib$a.so $(for s in $FIXED; do echo $OUT/$s.o; done) \
    $OUT/g$a.o $OUT/i${a}_*.o
done
rm -f $OUT/*.o
