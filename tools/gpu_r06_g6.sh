# dynamic range mode (batch-independent logits) re-measured: eager and graph-replayed forwards
for rep in 1 2; do
SMPQ_RANGE_MODE=dynamic timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 --warmup 10 > gpurun_out/r06_dyn.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_dyn.json')); print('dynamic rep $rep', d['value'], d['ms_per_step'], d['config']['range_mode'], d['config']['hip_graph'])" | tee -a gpurun_out/r06_dyn.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 40 --warmup 10 > gpurun_out/r06_sta.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_sta.json')); print('static rep $rep', d['value'], d['ms_per_step'], d['config']['range_mode'], d['config']['hip_graph'])" | tee -a gpurun_out/r06_dyn.txt
done
