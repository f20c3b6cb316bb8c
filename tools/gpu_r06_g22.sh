# more slices? SMPQ_STREAMS 2 / 3 / 4
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for cfg in "r50_mixed 256" "r34_4bit 512"; do set -- $cfg; for st in 2 3 4; do
SMPQ_STREAMS=$st timeout -k 10 200 python -u bench.py --no-cpu-baseline --config $1 --batch $2 > gpurun_out/r06_ab22.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab22.json')); print('$1 streams $st rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab22.txt
done; done; done
