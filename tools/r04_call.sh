# round-4 GPU session script (run from the repo root on the GPU box). Each step has its own time
# limit; the script stops at the first failure.
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval.py tests/test_gpu_driver.py -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04_evaltests.log 2>&1 || exit 2
timeout -k 10 300 python -u tools/eval_host_batches.py --out gpurun_out/r04_eval_host.json > gpurun_out/r04_eval_host.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py --layers > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err || exit 4
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -q -s --timeout 300 --timeout-method thread -k full_size > gpurun_out/r04_full_size_parity.log 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --config r18_u8 --no-cpu-baseline > gpurun_out/r04_bench_r18.json 2> gpurun_out/r04_bench_r18.err || exit 6
timeout -k 10 300 python -u bench.py --config r34_4bit --batch 512 --no-cpu-baseline > gpurun_out/r04_bench_r34.json 2> gpurun_out/r04_bench_r34.err || exit 7
