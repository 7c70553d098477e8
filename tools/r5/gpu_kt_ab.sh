# Same-box kernel-trace A/B of one switch on one workload: $1 = c2 | c4, $2 = VAR, $3 $4 = its two values, $5 = tag.
# Per-kernel summaries (tools/trace_summary.py) of each arm; optional PRETEST pytest node ids first.
set -e
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
w=$1
O=gpurun_out/r5kt_${5:-ab}
R=/tmp/r5kt_raw
mkdir -p $O $R
[ -n "$PRETEST" ] && { timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread $PRETEST > $O/pretest.log 2>&1 || { tail -40 $O/pretest.log; exit 1; }; tail -1 $O/pretest.log; }
if [ $w = c2 ]; then X="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4 --no-c5 --no-batch64"
else X="python3 bench.py --only-c4 --steps 1 --warmup 0 --no-timing"; fi
for v in $3 $4; do
  export $2=$v
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt_$v -- $X > $O/kt_${w}_$v.log 2>&1
  python3 tools/trace_summary.py $(find $R/kt_$v -name "*kernel_trace.csv" | head -1) > $O/${w}_${2}_$v.txt
  rm -rf $R/kt_$v
  head -12 $O/${w}_${2}_$v.txt
done
