# Same-box A/B of two builds of libsuta (SUTA_LIB): config C2 only; $1 = tag, $2 = the alternative library
set -e
O=gpurun_out/r4ablib
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
X="python bench.py --steps 2 --no-c4 --no-c5 --no-batch64 --no-split --no-cpu-baseline"
for i in 1 2; do
  for v in new alt; do
    if [ $v = alt ]; then export SUTA_LIB=$2; else unset SUTA_LIB; fi
    timeout -k 10 300 $X > $O/$1_$v.$i.json 2> $O/$1_$v.$i.err
    python -c "import json; d=json.loads(open('$O/$1_$v.$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['frac'], d['attention']['tflops'], d['time_breakdown_ms']['attention'])"
  done
done
