# Kernel trace of config C5 (512 TED-like utterances, one engine, eager per group) reduced by tools/trace_summary.py
set -e
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
O=gpurun_out/r5prof
R=/tmp/r5prof_raw_c5
mkdir -p $O $R
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -- python3 bench.py --only-c5 --no-timing --c5-engines 1 > $O/kt_c5.log 2>&1
python3 tools/trace_summary.py $(find $R/kt -name "*kernel_trace.csv" | head -1) > $O/c5_trace_summary.txt
cp $(find $R/kt -name "*kernel_stats.csv" | head -1) $O/c5_kernel_stats.csv
rm -rf $R
head -25 $O/c5_trace_summary.txt
