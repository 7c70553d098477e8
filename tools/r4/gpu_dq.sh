# dQ in-launch combination: parity (bitwise vs the reduce pass, fp32 and bf16 planes; flash parity suite) and
# same-box A/B of SUTA_DQ_INLAUNCH on C4 and C2
set -e
export TMPDIR=/tmp
O=gpurun_out/r4dq
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_large_bf16.py -k "dq_inlaunch or fused_delta" tests/test_gpu_parity.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for x in 1 0; do
    SUTA_DQ_INLAUNCH=$x timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_dq$x.$i.json 2> $O/c4_dq$x.$i.err
    python -c "import json; d=json.load(open('$O/c4_dq$x.$i.json')); print('c4 dq=$x', d['value'], d['roofline']['frac'], d['attention'])"
  done
done
for x in 1 0; do
  SUTA_DQ_INLAUNCH=$x timeout -k 10 300 python bench.py --steps 2 --no-c4 --no-c5 --no-batch64 --no-split --no-cpu-baseline > $O/c2_dq$x.json 2> $O/c2_dq$x.err
  python -c "import json; d=json.loads(open('$O/c2_dq$x.json').read().strip().splitlines()[-1]); print('c2 dq=$x', d['value'], d['roofline']['frac'], d['attention'])"
done
