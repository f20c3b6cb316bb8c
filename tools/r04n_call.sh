# round-4: shader-clock stamps of the LDS-DMA kernel (128x64 tile, BK 64) on short- and long-K R50 shapes
mkdir -p gpurun_out
: > gpurun_out/r04n_stamps.txt
for args in "lw1 64 256 1 56" "lw3 64 256 1 56" "lw1 256 64 1 56" "lw1 1024 256 1 14" "lw1 64 64 3 56" "lw1 256 256 3 14"; do
  set -- $args
  b=$1; shift
  echo "$b $*" >> gpurun_out/r04n_stamps.txt
  timeout -k 10 120 ./tools/bin/stamp_$b "$@" >> gpurun_out/r04n_stamps.txt 2>&1 || exit 2
done
