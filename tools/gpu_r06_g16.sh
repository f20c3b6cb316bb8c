# resident kernels with the per-image scales staged in LDS (no vmcnt wait inside the tile loop)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_pair.py tests/test_gpu_resident.py > gpurun_out/r06_tab_tests.log 2>&1 || { tail -50 gpurun_out/r06_tab_tests.log; exit 1; }
tail -1 gpurun_out/r06_tab_tests.log
for b in 128 256; do TB_BATCH=$b timeout -k 10 200 python -u tools/pair_bench.py 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_tab_pair.txt || exit 1; done
for pat in c1 c3 ds; do TB_BATCH=128 timeout -k 10 200 python -u tools/tile_bench.py 2,3,9,18,19,27,28,32,47,48,49,50 $pat >> gpurun_out/r06_tab_tiles_b128.txt 2>&1 || exit 1; done
grep -v amdgpu.ids gpurun_out/r06_tab_tiles_b128.txt
for rep in 1 2 3; do for v in "1 1" "0 1"; do set -- $v
SMPQ_FUSE_DS=$1 SMPQ_PAIR_1X1=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_ab16.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_ab16.json')); print('fuse_ds=$1 pair=$2 rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_ab16.txt
done; done
# stem: raw barrier (this build) vs __syncthreads (variants/stem_sync.so)
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu.py -k "fused_stem" 2>&1 | tail -1
for rep in 1 2; do
timeout -k 10 200 python -u tools/stem_microbench.py 256 3 30 2>&1 | grep -v amdgpu.ids | sed "s/^/new rep $rep: /" | tee -a gpurun_out/r06_stem_barrier.txt || exit 1
SMPQ_LIB=$PWD/variants/stem_sync.so timeout -k 10 200 python -u tools/stem_microbench.py 256 3 30 2>&1 | grep -v amdgpu.ids | sed "s/^/old rep $rep: /" | tee -a gpurun_out/r06_stem_barrier.txt || exit 1
done
