# Re-entry check of HEAD: GPU suite, smoke, default bench line (as the driver runs them).
set -e
export TMPDIR=/tmp
O=gpurun_out/r2w
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
echo done
