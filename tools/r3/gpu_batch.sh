# Batch-size sweep (utterances per engine call): tile-round fill of the M = B*T GEMM grids.  C2 and C4, two passes.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3batch
mkdir -p $O
for i in 1 2; do
for b in 64 96 128 160; do
timeout -k 10 300 python bench.py --batch $b --steps 3 --no-split --no-cpu-baseline --no-c4 > $O/c2_b$b.$i.json 2> $O/c2_b$b.$i.err
done
done
for b in 64 96 128; do
timeout -k 10 400 python bench.py --only-c4 --c4-batch $b --steps 2 > $O/c4_b$b.json 2> $O/c4_b$b.err
done
echo done
