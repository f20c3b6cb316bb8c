# fused strided downsamples (layers 2-3): parity, then bench A/B against layer1-only fusion
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pair.py > gpurun_out/r06_g23_tests.log 2>&1 || { tail -50 gpurun_out/r06_g23_tests.log; exit 1; }
tail -1 gpurun_out/r06_g23_tests.log
for rep in 1 2 3; do for v in "1 256" "1 128" "1 64"; do set -- $v
SMPQ_FUSE_DS=$1 SMPQ_FUSE_DS_MAX_CIN=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_ab23.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab23.json')); print('fuse_ds=$1 maxcin=$2 rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab23.txt
done; done
