# round-4: fused stem ablations (SMPQ_SP_DIAG 1 no MFMA, 2 no epilogue, 3 neither, 4 no operand reads from LDS; 8 phase stamps), B=256 L=3
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/r04w_stem.txt
for v in base 1 2 3 4 base; do
  if [ $v = base ]; then unset SMPQ_LIB; else export SMPQ_LIB=$PWD/variants/sp$v.so; fi
  timeout -k 10 120 python -u tools/stem_microbench.py 256 3 20 >> gpurun_out/r04w_stem.txt 2>&1 || exit 3
done
SMPQ_LIB=$PWD/variants/sp8.so STAMPS=1 timeout -k 10 120 python -u tools/stem_microbench.py 256 3 20 >> gpurun_out/r04w_stem.txt 2>&1 || exit 4
