# VROW halo tiles for the BasicBlock nets (R18 / R34): committed table vs VROW at 14^2 + 7^2 vs 7^2 only
for rep in 1 2; do for cfg in "r34_4bit 512" "r18_u8 256"; do set -- $cfg; for tab in committed vtab_vrow_14_7.json vtab_vrow_7.json; do
if [ $tab = committed ]; then T=""; else T="SMPQ_TILE_TABLE=$PWD/$tab"; fi
env $T timeout -k 10 200 python -u bench.py --no-cpu-baseline --config $1 --batch $2 > gpurun_out/r06_vrow.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_vrow.json')); print('$1 $tab rep $rep', d['value'], d['ms_per_step'], d['config']['tile_table']['hits'])" | tee -a gpurun_out/r06_vrow.txt
done; done; done
