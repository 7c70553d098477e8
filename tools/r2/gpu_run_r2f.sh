set -e
export TMPDIR=/tmp
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_bf16.py -x -q --timeout 300 --timeout-method thread > $O/bf16_tests.log 2>&1
timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_planes.json 2> $O/c4_planes.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -- python3 bench.py --only-c4 --steps 2 --no-timing > $O/kt_c4.log 2>&1
echo done
