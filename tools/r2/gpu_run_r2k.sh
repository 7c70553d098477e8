set -e
export TMPDIR=/tmp
O=gpurun_out/r2k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_bf16.py -k "fused_attention or longest or bf16_large or planes" -x -q --timeout 200 --timeout-method thread > $O/attn.log 2>&1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-split > $O/b.json 2>/dev/null
echo done
