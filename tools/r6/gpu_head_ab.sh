# bf16 flash backward: one workgroup per head (SUTA_FLASH_BWD_HEAD=1) vs per key block + reduce (=0), interleaved;
# bitwise checksums must agree; then a ragged check (T = 262, 49) and the fp32 line.  $1 = output tag
set -e
O=gpurun_out/r6${1:-headab}
mkdir -p $O
for r in 1 2 3; do for hd in 0 1; do
  echo -n "HEAD=$hd " >> $O/ab.txt
  SUTA_FLASH_BWD_HEAD=$hd timeout -k 10 120 ./tools/attn_bench 1 164 399 16 10 >> $O/ab.txt 2>&1
done; done
for T in 262 49 1874 256 257; do for hd in 0 1; do
  echo -n "HEAD=$hd " >> $O/ab.txt
  SUTA_FLASH_BWD_HEAD=$hd timeout -k 10 120 ./tools/attn_bench 1 24 $T 16 3 >> $O/ab.txt 2>&1
done; done
cat $O/ab.txt
