# Round-2 final evidence, part 1: GPU suite, smoke, full bench line (CPU baseline, split, C4), kernel traces.
set -e
export TMPDIR=/tmp
O=gpurun_out/prof2d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python3 bench.py --steps 2 --warmup 1 --no-split --no-cpu-baseline --no-timing --no-c4 > $O/kt.log 2>&1
echo done
