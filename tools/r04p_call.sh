# round-4: strided downsample convs vs the same convs on a pre-subsampled input (stride 1), best tile each
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/batch_scaling.py ds 256 > gpurun_out/r04p_ds.txt 2>&1 || exit 2
