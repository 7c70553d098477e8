# Round-3 counter evidence: SQ passes (A: stall/MFMA-busy, B: instruction mix) for the headline (C2) and
# C4 workloads, C4 FETCH/WRITE bytes, kernel traces of both.  Each pass its own run (gpurun rules); the raw
# per-dispatch CSVs are reduced on the box (tools/pmc_sq.py, tools/pmc_traffic.py, tools/trace_summary.py)
# and deleted, since they exceed what gpurun copies back.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3sq
R=/tmp/r3sq_raw
mkdir -p $O $R
B="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4"
C="python3 bench.py --only-c4 --steps 2 --no-timing"
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_CVT"
csv() { find $R/$1 -name "*counter_collection.csv" | head -1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/kt_c4 -- $C > $O/kt_c4.log 2>&1
python3 tools/trace_summary.py $(find $R/kt_c4 -name "*kernel_trace.csv" | head -1) > $O/c4_trace_summary.txt
cp $(find $R/kt_c4 -name "*kernel_stats.csv" | head -1) $O/c4_kernel_stats.csv
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $R/c4_sqa -- $C > $O/c4_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $R/c4_sqb -- $C > $O/c4_sqb.log 2>&1
python3 tools/pmc_sq.py $(csv c4_sqa) $(csv c4_sqb) --json $O/c4_sq.json > $O/c4_sq.txt
rm -rf $R/c4_sqa $R/c4_sqb $R/kt_c4
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $R/c2_sqa -- $B > $O/c2_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $R/c2_sqb -- $B > $O/c2_sqb.log 2>&1
python3 tools/pmc_sq.py $(csv c2_sqa) $(csv c2_sqb) --json $O/c2_sq.json > $O/c2_sq.txt
rm -rf $R/c2_sqa $R/c2_sqb
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/c4_fetch -- $C > $O/c4_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/c4_write -- $C > $O/c4_write.log 2>&1
python3 tools/pmc_traffic.py $(csv c4_fetch) $(csv c4_write) $O/pmc_traffic_c4.json > $O/pmc_traffic_c4.txt
rm -rf $R
cat $O/c4_sq.txt $O/c2_sq.txt | head -60
echo done
