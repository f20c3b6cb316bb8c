# round-4 (second session) GPU script: batch scaling of the R50 conv shapes + HEAD layer table
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/batch_scaling.py all 32,64,128,256 > gpurun_out/r04b_batch_scaling.txt 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --layers --no-cpu-baseline > gpurun_out/r04b_bench.json 2> gpurun_out/r04b_bench.err || exit 3
