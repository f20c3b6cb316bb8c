# bench A/B: tile table with the generalized weight-stationary 1x1 tiles (committed) vs the previous
# table (variants/tiles_before_res1x1.json), R50 mixed B=256; then the R18/R34 downsample tiles
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do for tab in committed variants/tiles_before_res1x1.json; do
if [ $tab = committed ]; then T=""; else T="SMPQ_TILE_TABLE=$PWD/$tab"; fi
env $T timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_res1x1_ab.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_res1x1_ab.json')); print('$tab rep $rep', d['value'], d['ms_per_step'], d['config']['tile_table']['sha16'])" | tee -a gpurun_out/r06_res1x1_ab.txt
done; done
for b in 256; do TB_BATCH=$b timeout -k 10 200 python -u tools/tile_bench.py all ds18 >> gpurun_out/r06_res_tiles_ds18.txt 2>&1 || exit 1; done
cat gpurun_out/r06_res_tiles_ds18.txt
