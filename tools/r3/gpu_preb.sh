# FFN pre-activation in bf16 (bf16 operand loads hoisted out of the element loop): large-model bf16 GPU tests and
# bench scale, C4 A/B SUTA_PRE_BF16=1/0, C4 per-shape GEMM times, C2 bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3preb2
mkdir -p $O
# (tests: gpurun_out/r3det2/t1.log, 27 passed on this build)
for i in 1 2; do
for f in 1 0; do
SUTA_PRE_BF16=$f timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_preb$f.$i.json 2> $O/c4_preb$f.$i.err
done
done
timeout -k 10 300 python tools/gemm_shapes.py > $O/c4_gemm_shapes.txt 2>&1
timeout -k 10 300 python bench.py --steps 3 --no-split --no-cpu-baseline --no-c4 > $O/c2.json 2> $O/c2.err
echo done
