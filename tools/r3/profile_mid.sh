# Mid-round evidence on HEAD: kernel traces (C2, C4), SQ passes (C2, C4), PMC FETCH/WRITE (C2 with per-grid
# GEMM breakdown, C4); raw CSVs reduced on the box and deleted.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3mid
R=/tmp/r3mid_raw
mkdir -p $O $R
B="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4"
C="python3 bench.py --only-c4 --steps 1 --no-timing"
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_CVT"
csv() { find $R/$1 -name "*counter_collection.csv" | head -1; }
for w in c2 c4; do
  if [ $w = c2 ]; then X="$B"; else X="$C"; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt_$w -- $X > $O/kt_$w.log 2>&1
  python3 tools/trace_summary.py $(find $R/kt_$w -name "*kernel_trace.csv" | head -1) > $O/${w}_trace_summary.txt
  cp $(find $R/kt_$w -name "*kernel_stats.csv" | head -1) $O/${w}_kernel_stats.csv
  timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $R/${w}_sqa -- $X > $O/${w}_sqa.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $R/${w}_sqb -- $X > $O/${w}_sqb.log 2>&1
  python3 tools/pmc_sq.py $(csv ${w}_sqa) $(csv ${w}_sqb) --json $O/${w}_sq.json > $O/${w}_sq.txt
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/${w}_fetch -- $X > $O/${w}_fetch.log 2>&1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/${w}_write -- $X > $O/${w}_write.log 2>&1
  python3 tools/pmc_traffic.py $(csv ${w}_fetch) $(csv ${w}_write) $O/pmc_traffic_$w.json > $O/pmc_traffic_$w.txt
  python3 tools/pmc_traffic.py $(csv ${w}_fetch) $(csv ${w}_write) --by-grid > $O/pmc_traffic_${w}_by_grid.txt
  rm -rf $R/*
done
head -12 $O/c4_sq.txt
head -12 $O/c2_sq.txt
head -20 $O/pmc_traffic_c2_by_grid.txt
echo done
