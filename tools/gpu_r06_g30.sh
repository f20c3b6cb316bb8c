# halo 3x3 with a limb-plane residual (BasicBlock conv2): parity, single-launch timing of every config
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_halo.py > gpurun_out/r06_g30_tests.log 2>&1 || { tail -50 gpurun_out/r06_g30_tests.log; exit 1; }
tail -1 gpurun_out/r06_g30_tests.log
for b in 128 256; do
TB_BATCH=$b timeout -k 10 300 python -u tools/tile_bench.py 2,3,9,19,28,37,38,39,40,41,42,43,44,45,46 c2r_ > gpurun_out/r06_g30_tb$b.txt 2>&1 || { tail -30 gpurun_out/r06_g30_tb$b.txt; exit 1; }
grep c2r gpurun_out/r06_g30_tb$b.txt
done
