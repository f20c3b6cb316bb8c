# chains: fused downsample + weight offsets; parity then bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pair.py tests/test_gpu_resident.py > gpurun_out/r06_chain_tests.log 2>&1 || { tail -50 gpurun_out/r06_chain_tests.log; exit 1; }
tail -2 gpurun_out/r06_chain_tests.log
for rep in 1 2 3; do for v in "1 1" "0 1" "0 0"; do set -- $v
SMPQ_FUSE_DS=$1 SMPQ_PAIR_1X1=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_ab15.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab15.json')); print('fuse_ds=$1 pair=$2 rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab15.txt
done; done
