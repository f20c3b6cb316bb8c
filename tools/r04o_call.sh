# round-4: epilogue parameters staged in LDS before the K loop (new) vs loaded after it (prev), and prev with
# output tiles stored straight from registers (nostage): GPU tile/model tests on new, then bench A/B on one box
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_halo.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04o_tests.log 2>&1 || exit 2
: > gpurun_out/r04o_ab.txt
for rep in 1 2; do
for v in new prev nostage; do
  if [ $v = new ]; then unset SMPQ_LIB; else export SMPQ_LIB=variants/libsmpq_$v.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --layers > gpurun_out/r04o_$v.json 2> gpurun_out/r04o_$v.err || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/r04o_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> gpurun_out/r04o_ab.txt
done
done
