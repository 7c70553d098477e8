# C4 interleaved runs of several environment configurations: $1 = output tag, $2 = pytest selection ("" for none) with
# -k "$3", then one argument per configuration ("-" = defaults, else space-separated VAR=value pairs); 2 rounds
set -e
export TMPDIR=/tmp
O=gpurun_out/r6$1
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $2 -k "$3" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
shift 3
for r in 1 2; do
  i=0
  for c in "$@"; do
    i=$((i+1))
    if [ "$c" = "-" ]; then c=""; fi
    env $c timeout -k 10 300 python bench.py --only-c4 > $O/c$i.$r.json 2> $O/c$i.$r.err
    echo "c$i.$r [$c] $(python -c "import json,sys; d=json.loads(open('$O/c$i.$r.json').read().strip().splitlines()[-1]); tb=d['time_breakdown_ms']; print(d['value'], d['roofline']['frac'], 'gemm', tb['gemm'], 'attn', tb['attention'], 'norm', tb['norm'])")" | tee -a $O/summary.txt
  done
done
