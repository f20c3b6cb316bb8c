#!/bin/bash
# Round profile bundle (GPU box, repo root): PMC HBM traffic of the three bench configs (bound to
# this library / tile table, copied into profiles/ so the bench lines below attach them), the
# bench lines with CPU baselines and layer tables, a rocprofv3 kernel-trace --stats run of the
# default bench, and PMC instruction-mix / wave-state groups for R50 and R34.
# usage: bash tools/final_bundle.sh <tag>   -> gpurun_out/<tag>/...
set -o pipefail
export TMPDIR=/tmp
T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
step() { echo "[$(date +%T)] $*" | tee -a $O/steps.log; }
step pmc traffic r50
bash tools/pmc_traffic.sh r50_mixed 3 256 2 || exit 1
step pmc traffic r18
bash tools/pmc_traffic.sh r18_u8 3 256 2 || exit 1
step pmc traffic r34
bash tools/pmc_traffic.sh r34_4bit 3 512 2 || exit 1
cp gpurun_out/pmc_traffic_r50_mixed_L3_B256_S2.json gpurun_out/pmc_traffic_r18_u8_L3_B256_S2.json \
   gpurun_out/pmc_traffic_r34_4bit_L3_B512_S2.json profiles/ || exit 1
step bench r50
timeout -k 10 300 python3 -u bench.py --layers > $O/bench_r50_mixed.json 2> $O/bench_r50_mixed.err || exit 1
step bench r18
timeout -k 10 300 python3 -u bench.py --config r18_u8 --layers > $O/bench_r18_u8.json 2> $O/bench_r18_u8.err || exit 1
step bench r34
timeout -k 10 300 python3 -u bench.py --config r34_4bit --batch 512 --layers > $O/bench_r34_4bit_b512.json 2> $O/bench_r34_4bit_b512.err || exit 1
step rocprof stats
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
step pmc groups r50
bash tools/pmc_layers.sh $O/pmc_r50 || exit 1
step pmc groups r34
bash tools/pmc_layers.sh $O/pmc_r34 --config r34_4bit --batch 512 || exit 1
step done
