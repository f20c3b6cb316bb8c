set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_driver.py tests/test_gpu_eval.py tests/test_gpu_dp.py tests/test_gpu_mp.py > gpurun_out/r06_t1.log 2>&1 || { tail -30 gpurun_out/r06_t1.log; exit 1; }
tail -3 gpurun_out/r06_t1.log
for rep in 1 2; do for cfg in "r18_u8 256" "r34_4bit 512"; do set -- $cfg; for s in 1 2; do
timeout -k 10 200 python -u bench.py --no-cpu-baseline --config $1 --batch $2 --streams $s > gpurun_out/r06_s_$1_$s_$rep.json 2>/dev/null || exit 1
python -c "import json,sys; d=json.load(open('gpurun_out/r06_s_$1_$s_$rep.json')); print('$1 streams $s rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_streams.txt
done; done; done
