# Branch-free GELU / GELU' in the bf16-plane GEMM epilogues: large-model bf16 GPU tests and bench scale, C4 A/B
# SUTA_FAST_GELU=1/0, C4 per-shape GEMM times.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3fg
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_bf16.py tests/test_gpu_bench_scale.py -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for f in 1 0; do
SUTA_FAST_GELU=$f timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_fg$f.$i.json 2> $O/c4_fg$f.$i.err
done
done
timeout -k 10 300 python tools/gemm_shapes.py > $O/c4_gemm_shapes.txt 2>&1
echo done
