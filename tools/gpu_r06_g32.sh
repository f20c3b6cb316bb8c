# step A/B: fused downsample for layers 1-3 (MAX_CIN 256, default) vs layers 1-2 only (128)
set -o pipefail
mkdir -p gpurun_out
T=gpurun_out/r06_g32; mkdir -p $T
for rep in 1 2 3; do for v in 256 128; do
SMPQ_FUSE_DS_MAX_CIN=$v timeout -k 10 200 python3 -u bench.py --no-cpu-baseline > $T/out.json 2>$T/err.txt || { tail -20 $T/err.txt; exit 1; }
python3 -c "import json; d=json.load(open('$T/out.json')); print('max_cin $v rep $rep', d['value'], d['ms_per_step'])" | tee -a $T/ab.txt
done; done
