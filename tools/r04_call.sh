# round-4 GPU session script (run from the repo root on the GPU box): full GPU suite, tile-table tuning,
# host-batch evaluation loop, default bench. Each step has its own time limit; the script stops at the
# first GPU-side failure.
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r04_gputests3.log 2>&1
rc=$?
tail -6 gpurun_out/r04_gputests3.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u tools/tune_tiles.py --out gpurun_out/tiles_gfx950.json > gpurun_out/r04_tune.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/eval_host_batches.py --out gpurun_out/r04_eval_host.json > gpurun_out/r04_eval_host.log 2>&1 || exit 5
exit $rc
