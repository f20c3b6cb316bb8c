# round-4: batch slices on streams, A/B sweep on one box (alternating order, twice)
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/r04h_streams.txt
for s in 2 1 3 4 2 1 3 4; do
  timeout -k 10 200 python -u bench.py --streams $s --no-cpu-baseline > gpurun_out/r04h_s$s.json 2> gpurun_out/r04h_s$s.err || exit 2
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/r04h_s$s.json').read().strip().splitlines()[-1]); print($s, d['value'], d['ms_per_step'])" >> gpurun_out/r04h_streams.txt
done
