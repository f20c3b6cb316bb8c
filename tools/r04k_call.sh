# round-4: which halo tiles pay in the real forward: R34 B=512 and R50 B=256 with table variants, alternating, one box
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/r04k_ab.txt
for rep in 1 2; do
for t in new nohalo no7 no14; do
  if [ $t = new ]; then unset SMPQ_TILE_TABLE; else export SMPQ_TILE_TABLE=variants/tiles_$t.json; fi
  timeout -k 10 200 python -u bench.py --config r34_4bit --batch 512 --no-cpu-baseline > gpurun_out/r04k_r34_$t.json 2> gpurun_out/r04k_r34_$t.err || exit 2
  timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r04k_r50_$t.json 2> gpurun_out/r04k_r50_$t.err || exit 3
  python3 -c "
import json
for c in ('r34','r50'):
    d=json.loads(open('gpurun_out/r04k_%s_$t.json'%c).read().strip().splitlines()[-1]); print('$t', c, d['value'], d['ms_per_step'])" >> gpurun_out/r04k_ab.txt
done
done
