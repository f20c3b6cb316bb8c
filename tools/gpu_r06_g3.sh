# SMPQ_NT_MIN_MB sweep: limb-plane outputs at least this large are stored non-temporally
for rep in 1 2; do for nt in 64 100 160 320 100000; do
SMPQ_NT_MIN_MB=$nt timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_nt_$nt.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_nt_$nt.json')); print('nt_min_mb $nt rep $rep', d['value'], d['ms_per_step'])" | tee -a gpurun_out/r06_nt.txt
done; done
# eager forwards (no graph): downsample branch on a side stream inside the batch slices or not
for rep in 1 2; do for d in 0 1; do
SMPQ_GRAPH=0 SMPQ_DS_IN_SLICES=$d timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r06_dsin_$d.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/r06_dsin_$d.json')); print('eager ds_in_slices $d rep $rep', d['value'], d['ms_per_step'], d['roofline']['gpu_ms_per_step'])" | tee -a gpurun_out/r06_dsin.txt
done; done
