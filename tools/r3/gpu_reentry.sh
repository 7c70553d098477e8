# Re-entry check of HEAD on a fresh box: full GPU suite, smoke, default bench (C2 + split + C4 + CPU baseline).
set -e
export TMPDIR=/tmp
O=gpurun_out/r3re
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
echo done
