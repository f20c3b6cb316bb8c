# round-4: zero-C first K step (no accumulator zero moves): GPU tile tests, then bench A/B vs the previous library on one box
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu.py tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread -k "tile or lean or logits or kmajor or halo or stem or static or offset" > gpurun_out/r04m_tests.log 2>&1 || exit 2
: > gpurun_out/r04m_ab.txt
for rep in 1 2 3; do
for v in new head; do
  if [ $v = head ]; then export SMPQ_LIB=variants/libsmpq_head.so; else unset SMPQ_LIB; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r04m_$v.json 2> gpurun_out/r04m_$v.err || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/r04m_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> gpurun_out/r04m_ab.txt
done
done
