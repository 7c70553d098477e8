# Chained dQ (one launch per key block, no partials / reduce pass): bitwise tests, then a same-box C4 A/B (SUTA_DQ_CHAIN 0 / 1)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5dqchain
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  "tests/test_gpu_large_bf16.py::test_pipelined_bf16_flash_backward_bitwise" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 0 1; do
    SUTA_DQ_CHAIN=$v timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_dqc$v.$i.json 2> $O/c4_dqc$v.$i.err
    python -c "import json; d=json.load(open('$O/c4_dqc$v.$i.json')); print('C4 dqchain=$v', d['value'], d['roofline']['frac'], d['time_breakdown_ms'])"
  done
done
