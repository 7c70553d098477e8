# bf16-plane flash forward: bf16 GPU tests, then C4 A/B (SUTA_FLASH_FWD_PLANE=1/0, interleaved) and the
# headline bench (attention compiled in MFMA-VGPR form).
set -e
export TMPDIR=/tmp
O=gpurun_out/r3ffp
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_bf16.py tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for p in 1 0; do
SUTA_FLASH_FWD_PLANE=$p timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_plane$p.$i.json 2> $O/c4_plane$p.$i.err
done
done
timeout -k 10 400 python bench.py --steps 4 --no-split --no-cpu-baseline --no-c4 > $O/bench.json 2> $O/bench.err
echo done
