set -o pipefail
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py -k "stem or native or s2d" > gpurun_out/r06_t2.log 2>&1 || { tail -30 gpurun_out/r06_t2.log; exit 1; }
tail -3 gpurun_out/r06_t2.log
timeout -k 10 120 python -u tools/stem_microbench.py 256 3 30 2>&1 | tee gpurun_out/r06_stem_mb.txt
SMPQ_LIB=$PWD/varlib_read2.so timeout -k 10 120 python -u tools/stem_microbench.py 256 3 30 2>&1 | tee -a gpurun_out/r06_stem_mb.txt
timeout -k 10 120 python -u tools/stem_microbench.py 256 3 30 2>&1 | tee -a gpurun_out/r06_stem_mb.txt
for i in 1 2; do for pb in 16 12; do SMPQ_STEM_PIXEL_BYTES=$pb timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_stem_bench_$pb.json 2>/dev/null || exit 1; python -c "import json; d=json.load(open('gpurun_out/r06_stem_bench_$pb.json')); print('pb $pb', d['value'], d['ms_per_step'])"; done; done
