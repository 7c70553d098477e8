# tools/hb_bench alone (variants as compiled in); $1 = output tag
set -e
O=gpurun_out/r4hbb
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 ./tools/hb_bench 10 3 > $O/hb_bench_$1.log 2>&1 || { cat $O/hb_bench_$1.log; exit 1; }
grep -E "hbx|hb128" $O/hb_bench_$1.log
