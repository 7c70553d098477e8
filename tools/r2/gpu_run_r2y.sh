# hb8 A/B on config C4 (same box, interleaved) + bf16 GPU tests with the ping-pong kernel on.
set -e
export TMPDIR=/tmp
O=gpurun_out/r2y
mkdir -p $O
timeout -k 10 120 ./tools/hb_bench 20 > $O/hb_bench.log 2>&1
for i in 1 2; do
SUTA_HB8=0 timeout -k 10 300 python bench.py --only-c4 --steps 2 --no-timing > $O/c4_off_$i.json 2> $O/c4_off_$i.err
SUTA_HB8=1 timeout -k 10 300 python bench.py --only-c4 --steps 2 --no-timing > $O/c4_on_$i.json 2> $O/c4_on_$i.err
done
SUTA_HB8=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "bf16 or large or plane" > $O/gpu_tests_hb8.log 2>&1
echo done
