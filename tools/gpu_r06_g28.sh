# step-level A/B of layer-3/4 tile choices inside the graph (R50 mixed B=256, 2 slices of 128)
set -o pipefail
mkdir -p gpurun_out
T=gpurun_out/r06_g28; mkdir -p $T
S="128,14,1024,256,1,0 128,14,256,256,3,0 128,28,256,256,3,0 128,14,512,512,3,0 128,7,2048,512,1,0 128,7,512,512,3,0"
rules() { for s in $S; do echo -n "$s=$1 "; done; }
python3 tools/table_variant.py $T/B.json 128,14,256,256,3,0=45 || exit 1
python3 tools/table_variant.py $T/C.json 128,14,256,256,3,0=46 || exit 1
python3 tools/table_variant.py $T/D.json $(rules 19) || exit 1
python3 tools/table_variant.py $T/E.json $(rules 33) || exit 1
python3 tools/table_variant.py $T/F.json $(rules 9) || exit 1
for rep in 1 2; do for v in A B C D E F; do
if [ $v = A ]; then TT=semilayer-wise-mixed-precision-quantization_amd/smpq/data/tiles_gfx950.json; else TT=$T/$v.json; fi
SMPQ_TILE_TABLE=$TT timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > $T/$v.json.out 2>$T/$v.err || { tail -20 $T/$v.err; exit 1; }
python3 -c "import json; d=json.load(open('$T/$v.json.out')); print('$v rep $rep', d['value'], d['ms_per_step'], d['config'].get('tile_table', d.get('tile_table','')))" | tee -a $T/ab.txt
done; done
