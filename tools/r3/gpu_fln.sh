# fused conv-stack LayerNorm backward: large-model GPU tests, C4 A/B (SUTA_FUSED_CONV_LN=1/0)
set -e
export TMPDIR=/tmp
O=gpurun_out/r3fln
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_bf16.py -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for f in 1 0; do
SUTA_FUSED_CONV_LN=$f timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_fused$f.$i.json 2> $O/c4_fused$f.$i.err
done
done
echo done
