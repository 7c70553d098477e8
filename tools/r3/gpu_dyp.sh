# bf16 dy planes for the stable-LN backward + conv0's unused dz0 write dropped: GPU tests (large bf16, bench scale,
# parity), C4 A/B SUTA_DY_PLANES=1/0 at 64 and 164 utterances, C2 at 164 / 328 utterances per call.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3dyp
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_large_bf16.py tests/test_gpu_bench_scale.py tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for f in 1 0; do
SUTA_DY_PLANES=$f timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_dyp$f.$i.json 2> $O/c4_dyp$f.$i.err
done
done
SUTA_DY_PLANES=1 timeout -k 10 400 python bench.py --only-c4 --c4-batch 164 --steps 2 > $O/c4_b164.json 2> $O/c4_b164.err
for b in 164 328; do
timeout -k 10 400 python bench.py --batch $b --steps 3 --no-split --no-cpu-baseline --no-c4 > $O/c2_b$b.json 2> $O/c2_b$b.err
done
echo done
