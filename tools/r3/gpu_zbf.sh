# bf16 storage of the conv stack's z_i / da_i (SUTA_CONV_Z_BF16): full GPU suite, C4 A/B at 64 utterances, default bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3zbf
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for f in 1 0; do
SUTA_CONV_Z_BF16=$f timeout -k 10 300 python bench.py --only-c4 --c4-batch 64 --steps 2 > $O/c4_zbf$f.$i.json 2> $O/c4_zbf$f.$i.err
done
done
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
echo done
