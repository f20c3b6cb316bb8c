#!/bin/bash
# Round profile bundle (on the GPU box, from the repo root): rocprofv3 kernel-trace stats of the
# default bench, the per-launch layer table, and the PMC HBM-traffic passes (tools/pmc_traffic.sh).
# Outputs under gpurun_out/ (copy the summaries into profiles/ afterwards).
set -e
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_round -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_round.log 2>&1
timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --layers > gpurun_out/layers_round.log 2>&1
bash tools/pmc_traffic.sh r50_mixed 3 256 > gpurun_out/pmc_round.log 2>&1
