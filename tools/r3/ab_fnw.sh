# HEAD with peeled last key tiles in both flash forwards: GPU parity tests; C4 A/B of the 8-wave bf16-plane flash
# forward (SUTA_FLASH_FWD_NW=8 vs 4); C2 bench; then C2 GEMM traffic with band orders.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3fnw
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_bf16.py tests/test_gpu_bench_scale.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for w in 4 8; do
SUTA_FLASH_FWD_NW=$w timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_nw$w.$i.json 2> $O/c4_nw$w.$i.err
done
done
timeout -k 10 300 python bench.py --steps 3 --no-split --no-cpu-baseline --no-c4 > $O/c2.json 2> $O/c2.err
bash tools/r3/pmc_order.sh
echo done
