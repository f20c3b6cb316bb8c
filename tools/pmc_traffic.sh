#!/bin/bash
# HBM traffic of bench.py's quantized-conv launches: two rocprofv3 --pmc passes (FETCH_SIZE, then
# WRITE_SIZE — separate passes, as gfx950's TCC block cannot count both at once), then
# tools/pmc_traffic.py -> gpurun_out/pmc_traffic_<config>_L<limbs>_B<batch>_S<slices>.json (copy it into
# profiles/, where bench.py reads it; it is bound to the library build, tile table and launch layout).
# usage: tools/pmc_traffic.sh [config] [limbs] [batch] [slices]     (on the GPU box, from the repo root)
set -e
export TMPDIR=/tmp
CFG=${1:-r50_mixed}; L=${2:-3}; B=${3:-256}; S=${4:-2}
O=gpurun_out/pmc_traffic_${CFG}_L$L
mkdir -p $O
ARGS="--config $CFG --limbs $L --batch $B --streams $S --steps 2 --warmup 1 --no-cpu-baseline"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py $ARGS > $O/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py $ARGS > $O/write.log 2>&1
python3 tools/pmc_traffic.py $O/fetch $O/write gpurun_out/pmc_traffic_${CFG}_L${L}_B${B}_S$S.json $O/fetch.log  # copy into profiles/
