# gemm_hbx / gemm_hbp A/B: parity (bitwise in every epilogue form and main loop, fused delta, C4 layout census) and
# a same-box C4 A/B over SUTA_HBX_FORM=2 / 0
set -e
export TMPDIR=/tmp
O=gpurun_out/r4hbpab
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_large_bf16.py tests/test_gpu_bench_scale.py::test_c4_bench_layout_bf16 > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for i in 1 2; do
  for x in 2 0; do
    SUTA_HBX_FORM=$x timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_f$x.$i.json 2> $O/c4_f$x.$i.err
    python -c "import json; d=json.load(open('$O/c4_f$x.$i.json')); print('hbx_form=$x', d['value'], d['roofline']['frac'], d['time_breakdown_ms'])"
  done
done
