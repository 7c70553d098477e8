# Conv weight gradients on a side stream: bitwise tests, then a same-box C4 A/B (SUTA_CONV_DW_SIDE 0 / 1, two rounds)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5dwside
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  "tests/test_gpu_large_bf16.py::test_pipelined_bf16_flash_backward_bitwise" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 0 1; do
    SUTA_CONV_DW_SIDE=$v timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_dws$v.$i.json 2> $O/c4_dws$v.$i.err
    python -c "import json; d=json.load(open('$O/c4_dws$v.$i.json')); print('C4 dwside=$v', d['value'], d['roofline']['frac'], d['time_breakdown_ms'])"
  done
done
