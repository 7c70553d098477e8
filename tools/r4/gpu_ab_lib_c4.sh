# Same-box A/B of two builds of libsuta (SUTA_LIB) on config C4, interleaved twice; $1 = tag, $2 = the alternative
set -e
O=gpurun_out/r4ablibc4
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_large_bf16.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  for v in new alt; do
    if [ $v = alt ]; then export SUTA_LIB=$2; else unset SUTA_LIB; fi
    timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/$1_$v.$i.json 2> $O/$1_$v.$i.err
    python -c "import json; d=json.load(open('$O/$1_$v.$i.json')); print('$v', d['value'], d['roofline']['frac'], d['time_breakdown_ms']['norm'])"
  done
done
