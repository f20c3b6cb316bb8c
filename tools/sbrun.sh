#!/bin/bash
# Timing-only runs of tools/stamp_bench.hip builds (tools/bin/sb_lw<LW>_a<ABLATE>), one line per shape.
# usage: bash tools/sbrun.sh "<ablate values>"   (on the GPU box, from the repo root)
set -e
for a in ${1:-0}; do
  for s in "256 256 3 14 64 1" "1024 256 1 14 64 1" "128 128 3 28 64 1" "512 512 3 7 64 1" "256 64 1 56 64 1"; do
    timeout -k 10 60 ./tools/bin/sb_lw1_a$a $s
  done
done
