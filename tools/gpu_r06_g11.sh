# the chained Bottleneck pair: parity (unit + model), its time vs the two launches, bench A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pair.py tests/test_gpu_resident.py "tests/test_gpu.py::test_model_logits_vs_reference" > gpurun_out/r06_pair_tests.log 2>&1 || { tail -40 gpurun_out/r06_pair_tests.log; exit 1; }
tail -2 gpurun_out/r06_pair_tests.log
for b in 128 256; do TB_BATCH=$b timeout -k 10 200 python -u tools/pair_bench.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_pair_bench.txt || exit 1; done
for rep in 1 2 3; do for pair in 1 0; do
SMPQ_PAIR_1X1=$pair timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_pair_ab.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_pair_ab.json')); print('pair=$pair rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_pair_ab.txt
done; done
