# resident 1x1 tiles with the copy-out and the next DMA issued before a tile's MFMAs: parity + tile times
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_resident.py > gpurun_out/r06_res2_tests.log 2>&1 || { tail -30 gpurun_out/r06_res2_tests.log; exit 1; }
tail -2 gpurun_out/r06_res2_tests.log
for b in 128 256; do
  for pat in c1 c3 ds; do
    TB_BATCH=$b timeout -k 10 200 python -u tools/tile_bench.py ${CFGS:-2,3,9,12,18,19,22,27,28,32,47,48,49,50} $pat >> gpurun_out/r06_res2_tiles_b$b.txt 2>&1 || exit 1
  done
done
cat gpurun_out/r06_res2_tiles_b128.txt gpurun_out/r06_res2_tiles_b256.txt | grep -v amdgpu.ids
