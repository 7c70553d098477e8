# Env A/Bs on HEAD after the 32-bit epilogue.  hb_bench: bare C4 linears, 128x128 with 2 x 64-deep stages
# (default), 4 / 3 x 32-deep stages (ns 5 / 6), 256x256 ping-pong.  C4 loop: SUTA_HB_NS=2/5/6, SUTA_HB8=1.
# Headline: SUTA_GEMM_ORDER=0 (n fastest) vs 4 / 8 (bands of tile rows walked column by column).
set -e
export TMPDIR=/tmp
O=gpurun_out/r3ab
mkdir -p $O
timeout -k 10 200 ./tools/hb_bench 20 > $O/hb_bench.log 2>&1
for i in 1 2; do
for v in "SUTA_HB_NS=2" "SUTA_HB_NS=5" "SUTA_HB_NS=6" "SUTA_HB8=1"; do
env $v timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_$v.$i.json 2> $O/c4_$v.$i.err
done
for g in 0 4 8; do
SUTA_GEMM_ORDER=$g timeout -k 10 300 python bench.py --steps 3 --no-split --no-cpu-baseline --no-c4 > $O/c2_order$g.$i.json 2> $O/c2_order$g.$i.err
done
done
echo done
