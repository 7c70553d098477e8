# bf16 flash-backward diagnostic forms (tools/ab/attn_bench_diag, SUTA_FB_DIAG bits; wrong results): where the tile
# body's time goes; then a kernel trace of the default form.  $1 = output tag
set -e
export TMPDIR=/tmp
O=gpurun_out/r6${1:-fbdiag}
mkdir -p $O
for d in ${DGS:-0 1 2 4 8 16 32 64 128 63 127 191 255 0}; do
  echo -n "DG=$d  " >> $O/diag.txt
  SUTA_FB_DIAG=$d timeout -k 10 120 ./tools/ab/attn_bench_diag 1 164 399 16 10 >> $O/diag.txt 2>&1
done
cat $O/diag.txt
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r6kt -- ./tools/attn_bench 1 164 399 16 10 > $O/kt.log 2>&1
cp $(find /tmp/r6kt -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
cut -d, -f1-8 $O/kernel_stats.csv | head -12
