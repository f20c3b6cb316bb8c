# round-4: compile-time lean variant without ReLU / residual (downsample convs): GPU tests, bench A/B vs prev
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_dp.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04r_tests.log 2>&1 || exit 2
: > gpurun_out/r04r_ab.txt
for rep in 1 2 3; do
for v in new prev; do
  if [ $v = new ]; then unset SMPQ_LIB; else export SMPQ_LIB=variants/libsmpq_$v.so; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --layers > gpurun_out/r04r_$v.json 2> gpurun_out/r04r_$v.err || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/r04r_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> gpurun_out/r04r_ab.txt
done
done
