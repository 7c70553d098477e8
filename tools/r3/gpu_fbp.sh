# bf16-plane flash backward: bf16 GPU tests, C4 A/B (SUTA_FLASH_BWD_PLANE=1/0), SQ passes of C4 (new kernels)
set -e
export TMPDIR=/tmp
O=gpurun_out/r3fbp
R=/tmp/r3fbp_raw
mkdir -p $O $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_bf16.py -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
for i in 1 2; do
for p in 1 0; do
SUTA_FLASH_BWD_PLANE=$p timeout -k 10 300 python bench.py --only-c4 --steps 2 > $O/c4_bwdplane$p.$i.json 2> $O/c4_bwdplane$p.$i.err
done
done
C="python3 bench.py --only-c4 --steps 1 --no-timing"
SQA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
SQB="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_VALU_CVT"
csv() { find $R/$1 -name "*counter_collection.csv" | head -1; }
timeout -s KILL 200 rocprofv3 --pmc $SQA --output-format csv -d $R/sqa -- $C > $O/sqa.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc $SQB --output-format csv -d $R/sqb -- $C > $O/sqb.log 2>&1
python3 tools/pmc_sq.py $(csv sqa) $(csv sqb) --json $O/c4_sq.json > $O/c4_sq.txt
rm -rf $R
head -14 $O/c4_sq.txt
echo done
