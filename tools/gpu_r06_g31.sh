# step A/B: BasicBlock conv2 (3x3 + limb-plane residual) on the halo tiles vs the committed choices
set -o pipefail
mkdir -p gpurun_out
T=gpurun_out/r06_g31; mkdir -p $T
python3 tools/table_variant.py $T/V1.json 128,56,64,64,3,1=42 128,28,128,128,3,1=41 128,14,256,256,3,1=46 256,56,64,64,3,1=42 || exit 1
python3 tools/table_variant.py $T/V2.json 128,56,64,64,3,1=42 128,28,128,128,3,1=41 128,14,256,256,3,1=46 256,56,64,64,3,1=42 256,14,256,256,3,1=46 || exit 1
for rep in 1 2; do for cfg in r18_u8 r34_4bit; do for v in A V1 V2; do
if [ $v = A ]; then TT=semilayer-wise-mixed-precision-quantization_amd/smpq/data/tiles_gfx950.json; else TT=$T/$v.json; fi
if [ $cfg = r34_4bit ]; then X="--batch 512"; else X=""; fi
SMPQ_TILE_TABLE=$TT timeout -k 10 200 python3 -u bench.py --config $cfg $X --no-cpu-baseline > $T/out.json 2>$T/err.txt || { tail -20 $T/err.txt; exit 1; }
python3 -c "import json; d=json.load(open('$T/out.json')); print('$cfg $v rep $rep', d['value'], d['ms_per_step'], d['config'].get('tile_table', d.get('tile_table',''))['autotuned'])" | tee -a $T/ab.txt
done; done; done
