set -e
for b in sb_lw1_a0 sb_lw1_a64; do
  timeout -k 10 60 ./tools/bin/$b 256 256 3 14 64 1
  timeout -k 10 60 ./tools/bin/$b 1024 256 1 14 64 1
  timeout -k 10 60 ./tools/bin/$b 128 128 3 28 64 1
  timeout -k 10 60 ./tools/bin/$b 256 64 1 56 64 1
done
for b in sb_lw3_a0 sb_lw3_a64; do
  timeout -k 10 60 ./tools/bin/$b 1024 2048 1 14 64 2
  timeout -k 10 60 ./tools/bin/$b 512 1024 1 28 64 2
  timeout -k 10 60 ./tools/bin/$b 256 512 1 56 64 2
done
