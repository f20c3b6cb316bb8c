set -e
for mb in 100000 0 64 160 400; do
  echo "NT_MIN_MB=$mb"; SMPQ_NT_MIN_MB=$mb timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 30 2>/dev/null | python3 -c "import sys,json; d=json.loads(sys.stdin.readlines()[-1]); print(d['value'], d['roofline']['conv_ms_per_step'])"
done
