# 32-bit-offset GEMM epilogue: GPU parity tests, then A/B (SUTA_EPI_FAST=1/0) on C4 and the headline.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3epi
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for f in 1 0; do
SUTA_EPI_FAST=$f timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_fast$f.$i.json 2> $O/c4_fast$f.$i.err
SUTA_EPI_FAST=$f timeout -k 10 300 python bench.py --steps 3 --no-split --no-cpu-baseline --no-c4 > $O/c2_fast$f.$i.json 2> $O/c2_fast$f.$i.err
done
done
echo done
