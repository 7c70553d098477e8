set -e
export TMPDIR=/tmp
O=gpurun_out/r2n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-split > $O/b.json 2> $O/b.err
echo done
