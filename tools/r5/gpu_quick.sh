# Quick check after a kernel change: the flash-kernel GPU tests, then one C2 and one C4 bench line; $1 = tag
set -e
export TMPDIR=/tmp
O=gpurun_out/r5q_${1:-q}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu -k "flash or fused_attention or bench_layout or pipelined or oracle" tests > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-c4 --no-c5 --no-batch64 --no-split --no-cpu-baseline --steps 4 > $O/c2.json 2> $O/c2.err
python -c "import json; d=json.load(open('$O/c2.json')); print('C2', d['value'], d['roofline']['frac'], 'attn', d['attention']['tflops'], d['attention']['ms'])"
timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4.json 2> $O/c4.err
python -c "import json; d=json.load(open('$O/c4.json')); print('C4', d['value'], d['roofline']['frac'], 'attn', d['attention']['tflops'], d['attention']['ms'])"
