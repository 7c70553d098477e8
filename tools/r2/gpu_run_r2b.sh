set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2b
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_attention or longest or graph_replay" -x -v --timeout 200 --timeout-method thread > gpurun_out/r2b/attn_tests.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2b/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r2b/bench.json 2> gpurun_out/r2b/bench.err
echo done
