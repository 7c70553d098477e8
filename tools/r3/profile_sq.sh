# Round-3 counter evidence: SQ passes (A: stall/MFMA-busy, B: instruction mix) for the headline (C2) and
# C4 workloads, C4 FETCH/WRITE bytes, kernel traces of both.  Each pass its own run (gpurun rules).
set -e
export TMPDIR=/tmp
O=gpurun_out/r3sq
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4"
C="python3 bench.py --only-c4 --steps 2 --no-timing"
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_CVT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -- $C > $O/kt_c4.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/c4_sqa -- $C > $O/c4_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/c4_sqb -- $C > $O/c4_sqb.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $O/c2_sqa -- $B > $O/c2_sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $O/c2_sqb -- $B > $O/c2_sqb.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/c4_fetch -- $C > $O/c4_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/c4_write -- $C > $O/c4_write.log 2>&1
echo done
