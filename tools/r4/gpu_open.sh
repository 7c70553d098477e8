# Round-4 opening run: the GPU suite (bench-layout pins at 164, two-rank bench, minimal-length ragged utterance),
# the default bench line (C2 + batch64 + split + C4 + C5 + CPU baseline) and smoke.  A heartbeat line per minute
# keeps the call visibly alive while bench.py computes.
set -e
export TMPDIR=/tmp
O=gpurun_out/r4open
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json | head -c 600
echo done
