# round-4 final bundle: default bench (CPU baseline), R18 / R34 lines, rocprofv3 kernel-trace stats, layer table, PMC traffic
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 120 ./tools/bin/stream_bench > gpurun_out/r04t_stream.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_halo.py -x -q --timeout 200 --timeout-method thread -k model > gpurun_out/r04t_halo_model.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r04t_bench.json 2> gpurun_out/r04t_bench.err || exit 2
timeout -k 10 300 python -u bench.py --config r18_u8 --no-cpu-baseline > gpurun_out/r04t_bench_r18.json 2> gpurun_out/r04t_bench_r18.err || exit 3
timeout -k 10 300 python -u bench.py --config r34_4bit --batch 512 --no-cpu-baseline > gpurun_out/r04t_bench_r34.json 2> gpurun_out/r04t_bench_r34.err || exit 4
bash tools/profile_round.sh || exit 5
