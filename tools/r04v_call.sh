# round-4: batch slices started with a skew (slice 1 waits for slice 0's first k stages), same-box bench A/B
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/r04v_ab.txt
for rep in 1 2; do
for k in 0 1 2 4 8; do
  SMPQ_SLICE_SKEW=$k timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r04v_$k.json 2> gpurun_out/r04v_$k.err || exit 3
  python3 -c "import json; d=json.loads(open('gpurun_out/r04v_$k.json').read().strip().splitlines()[-1]); print('r50 skew $k', d['value'], d['ms_per_step'])" >> gpurun_out/r04v_ab.txt
done
done
