set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2a
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2a/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r2a/bench.json 2> gpurun_out/r2a/bench.err
timeout -k 10 300 python tools/bench_graphs.py > gpurun_out/r2a/graphs.log 2>&1
echo done
