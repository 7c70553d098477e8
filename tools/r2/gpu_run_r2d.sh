set -e
export TMPDIR=/tmp
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_bf16.py -k "fused_attention or longest or bf16_large or base_suta or tiny_suta" -x -q --timeout 200 --timeout-method thread > $O/attn_tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python3 bench.py --steps 1 --warmup 1 --no-split --no-cpu-baseline --no-timing --no-c4 > $O/kt.log 2>&1
echo done
