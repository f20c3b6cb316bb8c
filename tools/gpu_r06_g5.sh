# bench length: default (20 steps, 5 warm-up) vs longer runs (clock ramp / steady state)
for rep in 1 2; do for sw in "20 5" "100 30" "300 30"; do set -- $sw
timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps $1 --warmup $2 > gpurun_out/r06_len.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_len.json')); print('steps $1 warmup $2 rep $rep', d['value'], d['ms_per_step'], d['roofline']['gpu_ms_per_step'])" | tee -a gpurun_out/r06_len.txt
done; done
