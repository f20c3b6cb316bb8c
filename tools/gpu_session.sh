#!/bin/bash
# One GPU session on the MI355X box (run from the repo root through gpurun), replacing the per-call
# wrapper scripts of earlier rounds:
#
#   bash tools/gpu_session.sh <tag> <step> [<step> ...]
#
# Named steps (each under its own time limit, output in gpurun_out/<tag>_<step>.*):
#   gputests   pytest -m gpu (whole suite)        smoke      __graft_entry__.smoke()
#   bench      default bench line + layer table    r18 / r34  the other bench configs
#   trace      rocprofv3 kernel trace of the default bench (+ summary, graph-region timeline)
#   traffic    PMC FETCH/WRITE passes (tools/pmc_traffic.sh)   parity  full-size parity tests
#   pmc        PMC screen of every conv launch + per-group summary (tools/pmc_layers.sh)
# Any other argument (it must contain a space) is run as a command with a 600 s limit.
# The session stops at the first failing step (no GPU work after a fault, abort or time-out).
set -u
ncmd=0
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
tag=$1
shift
mkdir -p gpurun_out
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -rf"
run() {  # run <limit_s> <log> <command...>
  local lim=$1 log=$2
  shift 2
  echo "[$(date +%T)] $tag: $*"
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  echo "[$(date +%T)] rc=$rc ($log)"
  tail -3 "$log"
  [ $rc -eq 0 ] || exit $rc
}
for step in "$@"; do
  o=gpurun_out/${tag}_${step}
  case "$step" in
    gputests) run 900 $o.log $PYT tests -m gpu ;;
    smoke) run 300 $o.log python -u -c "import __graft_entry__ as g; g.build(); g.smoke()" ;;
    bench) run 300 $o.json sh -c "python -u bench.py --layers 2> $o.err" ;;
    r18) run 300 $o.json sh -c "python -u bench.py --config r18_u8 --no-cpu-baseline --layers 2> $o.err" ;;
    r34) run 300 $o.json sh -c "python -u bench.py --config r34_4bit --batch 512 --no-cpu-baseline --layers 2> $o.err" ;;
    trace)
      run 300 $o.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
        python3 bench.py --no-cpu-baseline
      f=$(find gpurun_out/${tag}_prof -name run_kernel_stats.csv | head -n 1)
      t=$(find gpurun_out/${tag}_prof -name run_kernel_trace.csv | head -n 1)
      python tools/rocprof_summary.py "$f" "$t" 106 > $o.summary.txt 2>&1
      python tools/graph_region.py "$t" > $o.graph.txt 2>&1
      ;;
    traffic) run 600 $o.log bash tools/pmc_traffic.sh r50_mixed 3 256 ;;
    parity) run 600 $o.log $PYT tests/test_gpu.py -m gpu -s -k full_size ;;
    pmc) run 900 $o.log bash tools/pmc_layers.sh gpurun_out/${tag}_pmc ;;
    *" "*) run 600 gpurun_out/${tag}_cmd$((++ncmd)).log bash -c "$step" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$(date +%T)] $tag: all steps ok"
