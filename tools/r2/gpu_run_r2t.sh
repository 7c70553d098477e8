set -e
export TMPDIR=/tmp
O=gpurun_out/r2t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_bf16.py -x -v -k "posconv or large_tracks" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4.json 2> $O/c4.err
echo done
