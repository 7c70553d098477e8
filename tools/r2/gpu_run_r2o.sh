set -e
export TMPDIR=/tmp
O=gpurun_out/r2o
mkdir -p $O
for s in 0 1 2 3 4 5 6; do
  timeout -k 10 60 ./tools/gemm_bench 0 1 $s >> $O/gb0.log 2>&1
  SUTA_GEMM_ORDER=1 timeout -k 10 60 ./tools/gemm_bench 0 1 $s >> $O/gb1.log 2>&1
done
timeout -k 10 120 ./tools/hb_bench 20 > $O/hb0.log 2>&1
SUTA_GEMM_ORDER=1 timeout -k 10 120 ./tools/hb_bench 20 > $O/hb1.log 2>&1
echo done
