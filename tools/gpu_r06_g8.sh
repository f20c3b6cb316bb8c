# resident 1x1 tiles, generalized (K 64..1024, slab 64/128/256, limb-plane residual): parity, then
# single-launch times of every 1x1 R50 shape at the in-graph slice batch (128) and at 256
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resident.py > gpurun_out/r06_res_tests.log 2>&1 || { tail -30 gpurun_out/r06_res_tests.log; exit 1; }
tail -3 gpurun_out/r06_res_tests.log
for b in 128 256; do
  for pat in c1 c3 ds_; do
    TB_BATCH=$b timeout -k 10 200 python -u tools/tile_bench.py all $pat >> gpurun_out/r06_res_tiles_b$b.txt 2>&1 || exit 1
  done
done
cat gpurun_out/r06_res_tiles_b128.txt
