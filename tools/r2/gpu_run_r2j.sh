set -e
export TMPDIR=/tmp
O=gpurun_out/r2j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_cli.py -k ted -x -v --timeout 500 --timeout-method thread > $O/ted.log 2>&1
echo done
