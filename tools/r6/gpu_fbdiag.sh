# bf16 flash-backward diagnostic forms (tools/ab/attn_bench_diag, SUTA_FB_DIAG bits; wrong results): where the tile
# body's time goes.  $1 = output tag
set -e
O=gpurun_out/r6${1:-fbdiag}
mkdir -p $O
for d in 0 1 2 4 8 16 32 3 6 7 14 15 31 63 0; do
  echo -n "DG=$d  " >> $O/diag.txt
  SUTA_FB_DIAG=$d timeout -k 10 120 ./tools/ab/attn_bench_diag 1 164 399 16 10 >> $O/diag.txt 2>&1
done
cat $O/diag.txt
