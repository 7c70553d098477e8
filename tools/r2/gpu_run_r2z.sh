# hb8 with fragments read one phase ahead (SUTA_HB8_PF=1): microbench, C4 A/B, GPU test.
set -e
export TMPDIR=/tmp
O=gpurun_out/r2z
mkdir -p $O
timeout -k 10 120 ./tools/hb_bench 20 > $O/hb_bench.log 2>&1
SUTA_HB8_PF=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_large_bf16.py -x -v --timeout 300 --timeout-method thread -k hb8 > $O/gpu_test_hb8pf.log 2>&1
for i in 1 2; do
SUTA_HB8=0 timeout -k 10 300 python bench.py --only-c4 --steps 2 --no-timing > $O/c4_off_$i.json 2> $O/c4_off_$i.err
SUTA_HB8=1 SUTA_HB8_PF=1 timeout -k 10 300 python bench.py --only-c4 --steps 2 --no-timing > $O/c4_pf_$i.json 2> $O/c4_pf_$i.err
done
echo done
