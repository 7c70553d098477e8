# bf16 flash backward after a change: attn_bench (C4 shape x2, ragged edge shapes), diag sweep, then the flash-related
# GPU tests and a C4 bench line.  $1 = output tag
set -e
export TMPDIR=/tmp
O=gpurun_out/r6${1:-fbnew}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for r in 1 2; do timeout -k 10 120 ./tools/attn_bench 1 164 399 16 10 >> $O/ab.txt 2>&1; done
for T in 262 49 1874 257; do timeout -k 10 120 ./tools/attn_bench 1 24 $T 16 3 >> $O/ab.txt 2>&1; done
for d in ${DGS:-0 1 128 255}; do
  echo -n "DG=$d  " >> $O/ab.txt
  SUTA_FB_DIAG=$d timeout -k 10 120 ./tools/ab/attn_bench_diag 1 164 399 16 10 >> $O/ab.txt 2>&1
done
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large_bf16.py -k "flash or ragged_edges or large_tracks or hbx_slice" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --only-c4 > $O/c4.json 2> $O/c4.err
python - <<PY
import json
d = json.loads(open("$O/c4.json").read().strip().splitlines()[-1])
print("C4", d["value"], d["roofline"]["frac"], "attn", d["attention"]["tflops"], d["time_breakdown_ms"])
PY
