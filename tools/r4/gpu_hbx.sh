# bf16-plane GEMM main-loop A/B on the C4 linear shapes (tools/hb_bench: hb 128 x 128, hb8, hbx 32x32x16 / 16x16x32)
set -e
O=gpurun_out/r4hbx
mkdir -p $O
timeout -k 10 300 ./tools/hb_bench ${1:-10} ${2:-3} > $O/hb_bench${3}.log 2>&1 || { cat $O/hb_bench${3}.log; exit 1; }
cat $O/hb_bench${3}.log
