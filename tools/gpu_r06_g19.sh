# 1x1 shapes, every tile config, B=128 (slice) and 256, after the resident LDS-scale fix
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/r06_t19_b*.txt
for b in 128 256; do for pat in c1 c3 ds; do
TB_BATCH=$b timeout -k 10 300 python -u tools/tile_bench.py all $pat >> gpurun_out/r06_t19_b$b.txt 2>&1 || exit 1
done; done
echo done
