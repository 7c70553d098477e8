# Full GPU suite + smoke + default bench line (C2, batch64, split, C4, C5, CPU baseline); $1 = output tag
set -e
export TMPDIR=/tmp
O=gpurun_out/r6${1:-full}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -60 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
python - <<PY
import json
d = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
print("C2", d["value"], d["roofline"]["frac"], "attn", d["attention"]["tflops"], "b64", d["batch64"]["value"])
c4 = d["c4"]; print("C4", c4["value"], c4["roofline"]["frac"], "attn", c4["attention"]["tflops"], c4["time_breakdown_ms"])
c5 = d["c5"]; print("C5", c5["value"], c5["audio_s_per_s"], c5["padded_frame_fraction"], c5["roofline"]["frac"])
PY
