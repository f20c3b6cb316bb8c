# fused downsample with / without the chained conv1 vs none (LDS-staged scales build)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pair.py > gpurun_out/r06_g17_tests.log 2>&1 || { tail -50 gpurun_out/r06_g17_tests.log; exit 1; }
tail -1 gpurun_out/r06_g17_tests.log
for rep in 1 2 3; do for v in "1 1" "1 0" "0 1"; do set -- $v
SMPQ_FUSE_DS=$1 SMPQ_DS_PAIR=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_ab17.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab17.json')); print('fuse_ds=$1 ds_pair=$2 rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab17.txt
done; done
