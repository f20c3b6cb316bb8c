# round-4: 1x1 DMA fast path (channel chunk in soffset, no per-step bounds check): tile tests + same-box bench A/B
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "tile or lean or static or kmajor or offsets or limbs_and_edges or parity_full" > gpurun_out/r04u_tests.log 2>&1 || exit 1
: > gpurun_out/r04u_ab.txt
for rep in 1 2; do
for v in base new; do
  if [ $v = base ]; then export SMPQ_LIB=$PWD/variants/base.so; else unset SMPQ_LIB; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --layers > gpurun_out/r04u_$v$rep.json 2> gpurun_out/r04u_$v$rep.err || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/r04u_$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> gpurun_out/r04u_ab.txt
done
done
