# Round-6 evidence at the bench defaults (164 utterances per call): kernel trace + summary, two SQ passes and the
# FETCH / WRITE passes of one workload ($1 = c2 | c4); raw CSVs reduced on the box and deleted.
set -e
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
export SUTA_GRAPHS=0   # rocprofv3 --pmc crashes on a launched hipGraph (the timed call's capture); eager runs the same kernels
w=$1
O=gpurun_out/r6prof
R=/tmp/r6prof_raw_$w
mkdir -p $O $R
if [ $w = c2 ]; then X="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4 --no-c5 --no-batch64"
else X="python3 bench.py --only-c4 --steps 1 --warmup 0 --no-timing"; fi
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_CVT"
csv() { find $R/$1 -name "*counter_collection.csv" | head -1; }
if [ -z "$SKIPKT" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt -- $X > $O/kt_$w.log 2>&1
python3 tools/trace_summary.py $(find $R/kt -name "*kernel_trace.csv" | head -1) > $O/${w}_trace_summary.txt
cp $(find $R/kt -name "*kernel_stats.csv" | head -1) $O/${w}_kernel_stats.csv
rm -rf $R/kt
fi
timeout -s KILL 400 rocprofv3 --pmc $SQA --output-format csv -d $R/sqa -- $X > $O/${w}_sqa.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc $SQB --output-format csv -d $R/sqb -- $X > $O/${w}_sqb.log 2>&1
python3 tools/pmc_sq.py $(csv sqa) $(csv sqb) --json $O/${w}_sq.json > $O/${w}_sq.txt
rm -rf $R/sqa $R/sqb
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -- $X > $O/${w}_fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -- $X > $O/${w}_write.log 2>&1
python3 tools/pmc_traffic.py $(csv fetch) $(csv write) $O/pmc_traffic_$w.json > $O/pmc_traffic_$w.txt
python3 tools/pmc_traffic.py $(csv fetch) $(csv write) --by-grid > $O/pmc_traffic_${w}_by_grid.txt
rm -rf $R
echo done
