# Epilogue-class hb kernels (128 x 128): large-model bf16 GPU tests and bench scale, C4 A/B
# SUTA_HB_EPI_CLASS=1/0, C4 per-shape GEMM times.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3ec
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_bf16.py tests/test_gpu_bench_scale.py -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for f in 1 0; do
SUTA_HB_EPI_CLASS=$f timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_ec$f.$i.json 2> $O/c4_ec$f.$i.err
done
done
timeout -k 10 300 python tools/gemm_shapes.py > $O/c4_gemm_shapes.txt 2>&1
timeout -k 10 300 python bench.py --steps 3 --no-split --no-cpu-baseline --no-c4 > $O/c2.json 2> $O/c2.err
echo done
