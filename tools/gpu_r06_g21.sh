# batch slices per config again (after the resident / chain changes): SMPQ_STREAMS 1 vs 2
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for cfg in "r50_mixed 256" "r18_u8 256" "r34_4bit 512"; do set -- $cfg; for st in 2 1; do
SMPQ_STREAMS=$st timeout -k 10 200 python -u bench.py --no-cpu-baseline --config $1 --batch $2 > gpurun_out/r06_ab21.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab21.json')); print('$1 streams $st rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab21.txt
done; done; done
