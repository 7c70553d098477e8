set -e
export TMPDIR=/tmp
O=gpurun_out/r2u
mkdir -p $O
for g in 0 4 8 16; do
  echo "order $g" >> $O/hb.log
  SUTA_GEMM_ORDER=$g timeout -k 10 120 ./tools/hb_bench 20 >> $O/hb.log 2>&1
done
for g in 0 8; do
  for s in 0 1 2 4; do
    SUTA_GEMM_ORDER=$g timeout -k 10 60 ./tools/gemm_bench 0 1 $s >> $O/gb$g.log 2>&1
  done
done
echo done
