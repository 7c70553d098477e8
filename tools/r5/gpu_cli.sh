# Driver with several engines per GPU: the CLI GPU tests, then the C5 line at the driver's defaults (2 engines)
set -e
export TMPDIR=/tmp
O=gpurun_out/r5cli
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu tests/test_gpu_cli.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --only-c5 > $O/c5.json 2> $O/c5.err
python -c "import json; d=json.load(open('$O/c5.json')); print('C5', d['value'], d['audio_s_per_s'], d['padded_frame_fraction'], d['engines'], d['roofline']['frac'])"
