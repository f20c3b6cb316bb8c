# slice phase lag A/B (slice 1 forked after slice 0's first LAG blocks)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do for lag in -1 0 1 3 5 7 10 13; do
SMPQ_SLICE_LAG=$lag timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_lag.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_lag.json')); print('lag $lag rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_lag.txt
done; done
