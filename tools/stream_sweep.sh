#!/bin/bash
# Bench variants: serial vs concurrent downsample branch vs batch slices on streams (GPU box).
set -o pipefail
mkdir -p gpurun_out
b() { timeout -k 10 200 python3 -u bench.py --no-cpu-baseline "$@" > gpurun_out/sw.out 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; return 1; }
      grep '^{' gpurun_out/sw.out | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['ms_per_step'], d['config'].get('concurrent_downsample'), d['config'].get('batch_slices_on_streams'))"; }
SMPQ_CONCURRENT_DS=0 b --streams 1 && b --streams 1 && b --streams 2 && b --streams 3 && b --streams 4 && \
SMPQ_CONCURRENT_DS=0 b --streams 2 && b --streams 2 --batch 512
