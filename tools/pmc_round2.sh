#!/bin/bash
# Round-2 PMC screen of the best tile per shape (tools/pmc_shape.sh passes), then summaries.
set -e
mkdir -p gpurun_out/pmc2
bash tools/pmc_shape.sh 3 c2_256_256 30 gpurun_out/pmc2/c2_14
bash tools/pmc_shape.sh 3 c2_64_64 15 gpurun_out/pmc2/c2_56
bash tools/pmc_shape.sh 3 c1_1024_256 30 gpurun_out/pmc2/c1_14
bash tools/pmc_shape.sh 3 c3_64_256 34 gpurun_out/pmc2/c3_56
for s in c2_14 c2_56 c1_14 c3_56; do echo "== $s"; python3 tools/pmc_summary.py gpurun_out/pmc2/$s; done > gpurun_out/pmc2/summary.txt
