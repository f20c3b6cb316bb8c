#!/bin/bash
# Quick perf check after a kernel change: the GPU parity tests of the conv kernels, the
# microbench of the representative shapes on their tuned tiles, then the bench line.
set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/qp_tests.log 2>&1
timeout -k 10 200 python3 tools/conv_microbench.py 3 static "" 9,14,21,23,24,30 2>&1 | grep -v amdgpu > gpurun_out/qp_micro.log
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/qp_bench.log 2>&1
