# round-4: non-temporal store threshold A/B (SMPQ_NT_MIN_MB), alternating, on one box
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/r04i_nt.txt
for nt in 64 100000 16 64 100000 16; do
  SMPQ_NT_MIN_MB=$nt timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r04i_nt$nt.json 2> gpurun_out/r04i_nt$nt.err || exit 2
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04i_nt$nt.json').read().strip().splitlines()[-1]); print($nt, d['value'], d['ms_per_step'])" >> gpurun_out/r04i_nt.txt
done
