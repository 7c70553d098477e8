# Same-box A/Bs: SUTA_CONV_Z_BF16=1/0 on C4 (64 utterances), SUTA_FAST_GELU=1/0 on the headline (164 utterances).
set -e
export TMPDIR=/tmp
O=gpurun_out/r3ab2
mkdir -p $O
for i in 1 2; do
for f in 1 0; do
SUTA_CONV_Z_BF16=$f timeout -k 10 300 python bench.py --only-c4 --c4-batch 64 --steps 2 > $O/c4_zbf$f.$i.json 2> $O/c4_zbf$f.$i.err
SUTA_FAST_GELU=$f timeout -k 10 300 python bench.py --steps 2 --no-split --no-cpu-baseline --no-c4 > $O/c2_fg$f.$i.json 2> $O/c2_fg$f.$i.err
done
done
echo done
