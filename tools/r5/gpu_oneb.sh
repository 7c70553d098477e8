# One-barrier bf16 flash backward: its bitwise test, then a same-box C4 A/B (SUTA_FLASH_BWD_ONEB 0 / 1, interleaved, two
# rounds; bench.py --only-c4); $1 = tag
set -e
export TMPDIR=/tmp
O=gpurun_out/r5${1:-oneb}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  "tests/test_gpu_large_bf16.py::test_pipelined_bf16_flash_backward_bitwise" \
  "tests/test_gpu_parity.py::test_pipelined_fp32_flash_forward_bitwise" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 0 1; do
    SUTA_FLASH_BWD_ONEB=$v timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_oneb$v.$i.json 2> $O/c4_oneb$v.$i.err
    python -c "import json; d=json.load(open('$O/c4_oneb$v.$i.json')); print('C4 oneb=$v', d['value'], d['roofline']['frac'], 'attn', d['attention']['tflops'], d['time_breakdown_ms'])"
  done
done
