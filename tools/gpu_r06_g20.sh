# table 6d vs before, R50 and R18 (B=256) and R34 (B=512)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for cfg in "r50_mixed 256" "r18_u8 256" "r34_4bit 512"; do set -- $cfg; for tab in committed variants/tiles_before_6d.json; do
if [ $tab = committed ]; then T=""; else T="SMPQ_TILE_TABLE=$PWD/$tab"; fi
env $T timeout -k 10 200 python -u bench.py --no-cpu-baseline --config $1 --batch $2 > gpurun_out/r06_ab20.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab20.json')); print('$1 $tab rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab20.txt
done; done; done
