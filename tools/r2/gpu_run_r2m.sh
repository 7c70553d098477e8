set -e
export TMPDIR=/tmp
O=gpurun_out/r2m
mkdir -p $O
for s in 0 1 2 3 4 5 6; do
  SUTA_GEMM160=0 timeout -k 10 60 ./tools/gemm_bench 1 1 $s >> $O/gb.log 2>&1
  timeout -k 10 60 ./tools/gemm_bench 1 21 $s >> $O/gb.log 2>&1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_scale.py -x -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1
SUTA_GEMM160=0 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-split --no-c4 > $O/b0.json 2>/dev/null
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-split --no-c4 > $O/b1.json 2>/dev/null
echo done
