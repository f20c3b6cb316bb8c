# round-4: halo 3x3 kernel bring-up (bitwise tests, then per-shape timing with the halo tiles among the candidates)
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04c_halo_tests.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/batch_scaling.py c2_ 128,256 > gpurun_out/r04c_halo_scaling.txt 2>&1 || exit 3
