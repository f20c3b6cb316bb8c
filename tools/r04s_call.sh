# round-4: fused stem bands per CU (SMPQ_STEM_WG_PER_CU) A/B on one box
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/r04s_ab.txt
for rep in 1 2; do
for v in 1 2 3; do
  SMPQ_STEM_WG_PER_CU=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --layers > gpurun_out/r04s_$v.json 2> gpurun_out/r04s_$v.err || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/r04s_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> gpurun_out/r04s_ab.txt
  grep -A2 "launch  " gpurun_out/r04s_$v.err | tail -1 >> gpurun_out/r04s_ab.txt
done
done
