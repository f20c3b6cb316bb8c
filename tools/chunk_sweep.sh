#!/bin/bash
# images/s of bench.py over (chunk, streams): chunks of the batch round-robin over concurrent
# streams (engine._forward). Diagnostics; on the GPU box from the repo root.
set -e
mkdir -p gpurun_out
for cs in "256 2" "128 2" "64 2" "64 4" "32 2" "32 4" "128 4"; do
  set -- $cs
  timeout -k 10 150 python3 -u bench.py --no-cpu-baseline --roofline-steps 1 --chunk $1 --streams $2 > gpurun_out/sweep_$1_$2.log 2>&1
  echo "chunk $1 streams $2: $(grep '^{' gpurun_out/sweep_$1_$2.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
