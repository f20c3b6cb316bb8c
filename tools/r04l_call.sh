# round-4: per-launch instruction mix / wave states of the R50 forward (PMC)
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
bash tools/pmc_layers.sh gpurun_out/r04l_pmc_layers || exit 2
