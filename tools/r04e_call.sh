# round-4: halo kernel v2 (prologue diet, compile-time offsets, VGPR accumulators) + glds compile-time offsets
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_halo.py tests/test_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo or tile or lean or logits or kmajor" > gpurun_out/r04e_tests.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/batch_scaling.py c2_ 256 > gpurun_out/r04e_scaling.txt 2>&1 || exit 3
timeout -k 10 500 python -u tools/tune_tiles.py --out gpurun_out/r04e_tiles.json > gpurun_out/r04e_tune.log 2>&1 || exit 4
SMPQ_TILE_TABLE=gpurun_out/r04e_tiles.json timeout -k 10 300 python -u bench.py --layers --no-cpu-baseline > gpurun_out/r04e_bench.json 2> gpurun_out/r04e_bench.err || exit 5
timeout -k 10 300 python -u bench.py --layers --no-cpu-baseline > gpurun_out/r04e_bench_oldtable.json 2> gpurun_out/r04e_bench_oldtable.err || exit 6
