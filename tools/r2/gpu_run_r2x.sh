# hb8 (256x256 ping-pong bf16-plane GEMM) microbench + HEAD verification (suite, smoke, bench).
set -e
export TMPDIR=/tmp
O=gpurun_out/r2x
mkdir -p $O
timeout -k 10 120 ./tools/hb_bench 20 > $O/hb_bench.log 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
echo done
