# Round-2 profile set (run on the GPU box from the repo root): bench line, kernel traces (headline, C4),
# PMC traffic passes (headline; C4 with and without the bf16 planes) and one SQ stall pass (headline).
set -e
export TMPDIR=/tmp
O=gpurun_out/prof2
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4"
C="python3 bench.py --only-c4 --steps 2 --no-timing"
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python3 bench.py --steps 2 --warmup 1 --no-split --no-cpu-baseline --no-timing --no-c4 > $O/kt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -- $C > $O/kt_c4.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- $B > $O/pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- $B > $O/pmc_write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c4_fetch -- $C > $O/pmc_c4_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_c4_write -- $C > $O/pmc_c4_write.log 2>&1
SUTA_BF16_PLANES=0 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c4np_fetch -- $C > $O/pmc_c4np_fetch.log 2>&1
SUTA_BF16_PLANES=0 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_c4np_write -- $C > $O/pmc_c4np_write.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_sq -- $B > $O/pmc_sq.log 2>&1
echo done
