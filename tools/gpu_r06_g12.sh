# pair kernel: separate times; bench A/B pair all / layer1 only / off
set -o pipefail
mkdir -p gpurun_out
for b in 128 256; do TB_BATCH=$b timeout -k 10 200 python -u tools/pair_bench.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_pair_bench2.txt || exit 1; done
for rep in 1 2 3; do for v in "1 128" "1 64" "0 128"; do set -- $v
SMPQ_PAIR_1X1=$1 SMPQ_PAIR_MAX_CIN=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_pair_ab2.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_pair_ab2.json')); print('pair=$1 maxcin=$2 rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_pair_ab2.txt
done; done
