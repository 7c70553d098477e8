# Flash attention A/B: tools/ab/attn_bench_old vs tools/attn_bench (bf16 C4 shape, then fp32 C2 shape), interleaved;
# then (if $2) SQ passes of the new binary in mode $2; $1 = output tag
set -e
export TMPDIR=/tmp
O=gpurun_out/r6${1:-attnab}
R=/tmp/r6attn_raw
mkdir -p $O $R
for m in 1 0; do for r in 1 2; do
  echo -n "old " >> $O/ab.txt; timeout -k 10 120 ./tools/ab/attn_bench_old $m >> $O/ab.txt 2>&1
  echo -n "new " >> $O/ab.txt; timeout -k 10 120 ./tools/attn_bench $m >> $O/ab.txt 2>&1
done; done
cat $O/ab.txt
if [ -n "$2" ]; then
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE"
csv() { find $R/$1 -name "*counter_collection.csv" | head -1; }
NH=$([ "$2" = 1 ] && echo 16 || echo 12)
timeout -s KILL 120 rocprofv3 --pmc $SQA --output-format csv -d $R/sqa -- ./tools/attn_bench $2 164 399 $NH 3 > $O/sqa.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $SQB --output-format csv -d $R/sqb -- ./tools/attn_bench $2 164 399 $NH 3 > $O/sqb.log 2>&1
python3 tools/pmc_sq.py $(csv sqa) $(csv sqb) > $O/sq.txt
cat $O/sq.txt
fi
