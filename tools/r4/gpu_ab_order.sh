# C4 tile-order sweep (SUTA_GEMM_ORDER: unset = bands of 8 / 4 tile rows by grid width, G >= 2 = bands of G)
set -e
O=gpurun_out/r4order
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2; do
  for x in def 2 16; do
    if [ $x = def ]; then unset SUTA_GEMM_ORDER; else export SUTA_GEMM_ORDER=$x; fi
    timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_o$x.$i.json 2> $O/c4_o$x.$i.err
    python -c "import json; d=json.load(open('$O/c4_o$x.$i.json')); print('order=$x', d['value'], d['roofline']['frac'], d['time_breakdown_ms']['gemm'])"
  done
done
