# pair kernel times (no overflow); bench A/B: pair maxcin 128 / 64, and the ds table variant
set -o pipefail
mkdir -p gpurun_out
for b in 128 256; do TB_BATCH=$b timeout -k 10 200 python -u tools/pair_bench.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_pair_bench3.txt || exit 1; done
for rep in 1 2 3; do for v in "128 committed" "64 committed" "128 variants/tiles_ds6c.json" "64 variants/tiles_ds6c.json"; do set -- $v
if [ $2 = committed ]; then T=""; else T="SMPQ_TILE_TABLE=$PWD/$2"; fi
env $T SMPQ_PAIR_MAX_CIN=$1 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_ab14.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab14.json')); print('maxcin=$1 table=$2 rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab14.txt
done; done
