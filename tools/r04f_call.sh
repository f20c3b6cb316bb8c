# round-4: halo v3 (tiles per block, prefetch across tiles; pipelined tap fragments) A/B vs no tap pipelining
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04f_tests.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/batch_scaling.py c2_ 256 > gpurun_out/r04f_scaling_pipe.txt 2>&1 || exit 3
SMPQ_LIB=variants/libsmpq_nopipe.so timeout -k 10 300 python -u tools/batch_scaling.py c2_ 256 > gpurun_out/r04f_scaling_nopipe.txt 2>&1 || exit 4
