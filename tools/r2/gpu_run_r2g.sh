set -e
export TMPDIR=/tmp
O=gpurun_out/r2g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python tools/bf16_report.py > $O/bf16_report.log 2>&1
timeout -k 10 500 python bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo done
