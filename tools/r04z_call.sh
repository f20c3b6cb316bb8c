# round-4 final HEAD validation: full GPU suite, smoke, default bench line
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04z_gputests.log 2>&1 || exit 2
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/r04z_smoke.log 2>&1 || exit 3
timeout -k 10 300 python -u bench.py > gpurun_out/r04z_bench.json 2> gpurun_out/r04z_bench.err || exit 4
