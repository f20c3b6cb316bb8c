#!/bin/bash
# A/B of batch slices on streams (1 vs 2), alternating, on one GPU box.
set -o pipefail
mkdir -p gpurun_out
b() { timeout -k 10 200 python3 -u bench.py --no-cpu-baseline "$@" > gpurun_out/sw.out 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; return 1; }
      grep '^{' gpurun_out/sw.out | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$*', d['value'], d['ms_per_step'])"; }
for i in 1 2 3; do b --streams 1 --steps 40 && b --streams 2 --steps 40 || exit 1; done
