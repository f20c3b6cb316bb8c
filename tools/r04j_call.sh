# round-4: R34 B=512 / R18 B=256 with the earlier tile table vs the halo-era table, alternating, one box
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
: > gpurun_out/r04j_ab.txt
for rep in 1 2; do
for t in new old; do
  if [ $t = old ]; then export SMPQ_TILE_TABLE=variants/tiles_r04_old.json; else unset SMPQ_TILE_TABLE; fi
  timeout -k 10 200 python -u bench.py --config r34_4bit --batch 512 --no-cpu-baseline > gpurun_out/r04j_r34_$t.json 2> gpurun_out/r04j_r34_$t.err || exit 2
  timeout -k 10 200 python -u bench.py --config r18_u8 --no-cpu-baseline > gpurun_out/r04j_r18_$t.json 2> gpurun_out/r04j_r18_$t.err || exit 3
  python3 -c "
import json
for c in ('r34','r18'):
    d=json.loads(open('gpurun_out/r04j_%s_$t.json'%c).read().strip().splitlines()[-1]); print('$t', c, d['value'], d['ms_per_step'], d['config']['tile_table']['hits'], d['config']['tile_table']['autotuned'])" >> gpurun_out/r04j_ab.txt
done
done
