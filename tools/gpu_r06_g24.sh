# layer1 -> layer2 pair: parity, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pair.py > gpurun_out/r06_g24_tests.log 2>&1 || { tail -50 gpurun_out/r06_g24_tests.log; exit 1; }
tail -1 gpurun_out/r06_g24_tests.log
for rep in 1 2 3; do for v in new old; do
if [ $v = new ]; then L="SMPQ_PAIR_STAGE_ENTRY=1"; else L="SMPQ_PAIR_STAGE_ENTRY=0"; fi
env $L timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_ab24.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab24.json')); print('$v rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab24.txt
done; done
