# C4 A/B of an environment switch: interleaved bench.py --only-c4 runs with "$1" (e.g. SUTA_HBX_FORM=3) as "old" and
# the defaults as "new"; optional pytest selection first ($3, -k "$4"); outputs under gpurun_out/r6$2
set -e
export TMPDIR=/tmp
O=gpurun_out/r6${2:-envab}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
if [ -n "$3" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $3 -k "$4" > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for r in 1 2; do
  env $1 timeout -k 10 300 python bench.py --only-c4 > $O/old$r.json 2> $O/old$r.err
  timeout -k 10 300 python bench.py --only-c4 > $O/new$r.json 2> $O/new$r.err
done
python - <<PY
import json
for t in ("old1", "new1", "old2", "new2"):
    d = json.loads(open("$O/%s.json" % t).read().strip().splitlines()[-1])
    tb = d["time_breakdown_ms"]
    print(t, d["value"], d["roofline"]["frac"], "attn", d["attention"]["tflops"], "attn_ms", tb["attention"], "gemm", tb["gemm"], "norm", tb["norm"])
PY
