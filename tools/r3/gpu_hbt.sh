# conv weight gradients on bf16 planes (gemm_hbt_kernel) + fp32 band order: GPU tests (large bf16, bench scale,
# parity), C4 A/B SUTA_CONV_PLANES=1/0, C2 bench, C4 kernel trace.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3hbt
R=/tmp/r3hbt_raw
mkdir -p $O $R
timeout -k 10 800 python -u -m pytest tests/test_gpu_large_bf16.py tests/test_gpu_bench_scale.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for f in 1 0; do
SUTA_CONV_PLANES=$f timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_cpl$f.$i.json 2> $O/c4_cpl$f.$i.err
done
done
timeout -k 10 300 python bench.py --steps 3 --no-split --no-cpu-baseline --no-c4 > $O/c2.json 2> $O/c2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -- python3 bench.py --only-c4 --steps 1 --no-timing > $O/kt.log 2>&1
python3 tools/trace_summary.py $(find $R/kt -name "*kernel_trace.csv" | head -1) > $O/c4_trace_summary.txt
rm -rf $R
echo done
