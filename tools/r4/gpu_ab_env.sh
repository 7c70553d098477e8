# Same-box C4 A/B of one environment switch: $1 = variable, $2 $3 = the two values; plus the bf16 GPU tests
set -e
export TMPDIR=/tmp
O=gpurun_out/r4env_$1
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
[ -n "$NOTESTS" ] || timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_large_bf16.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
[ -n "$NOTESTS" ] || tail -1 $O/tests.log
for i in 1 2; do
  for x in $2 $3; do
    env $1=$x timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_$x.$i.json 2> $O/c4_$x.$i.err
    python -c "import json; d=json.load(open('$O/c4_$x.$i.json')); print('$1=$x', d['value'], d['roofline']['frac'], d['time_breakdown_ms']['norm'], d['attention']['ms'])"
  done
done
