# bench A/B: tile table with the weight-stationary downsample tile (committed) vs the previous table
for rep in 1 2 3; do for tab in committed vtab_old.json; do
if [ $tab = committed ]; then T=""; else T="SMPQ_TILE_TABLE=$PWD/$tab"; fi
env $T timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_res_ab.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_res_ab.json')); print('$tab rep $rep', d['value'], d['ms_per_step'], d['config']['tile_table']['sha16'])" | tee -a gpurun_out/r06_res_ab.txt
done; done
