# round-4: PMC screen of the halo 3x3 tiles vs the implicit-GEMM tiles
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/pmc_tiles.sh 3,37,38,43 c2_64_64_56 gpurun_out/r04d_pmc_c2_64 || exit 2
bash tools/pmc_tiles.sh 7,18,45 c2_256_256_14 gpurun_out/r04d_pmc_c2_256 || exit 3
