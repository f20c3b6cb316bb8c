# round-4: fused stem, parity 1 issues the next rows' DMA after its epilogue instead of before: stem tests, stem microbench + bench A/B
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "stem or pool or model_logits" > gpurun_out/r04y_tests.log 2>&1 || exit 1
: > gpurun_out/r04y_ab.txt
for rep in 1 2; do
for v in base new; do
  if [ $v = base ]; then export SMPQ_LIB=$PWD/variants/base.so; else unset SMPQ_LIB; fi
  timeout -k 10 120 python -u tools/stem_microbench.py 256 3 20 >> gpurun_out/r04y_ab.txt 2>&1 || exit 2
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r04y_$v$rep.json 2> gpurun_out/r04y_$v$rep.err || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/r04y_$v$rep.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> gpurun_out/r04y_ab.txt
done
done
