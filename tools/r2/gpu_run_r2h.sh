set -e
export TMPDIR=/tmp
O=gpurun_out/r2h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_attention or longest" -x -q --timeout 200 --timeout-method thread > $O/attn8.log 2>&1
SUTA_FLASH_BWD_NW=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_attention or longest" -x -q --timeout 200 --timeout-method thread > $O/attn4.log 2>&1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-split --no-c4 > $O/b8.json 2>/dev/null
SUTA_FLASH_BWD_NW=4 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-split --no-c4 > $O/b4.json 2>/dev/null
echo done
