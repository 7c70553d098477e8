# Second half of the round-2 profile set: C4 traffic with / without bf16 planes at 16 utterances per call
# (PMC passes serialise every dispatch; the 64-utterance no-plane pass outlived the box's silence limit)
# and the SQ stall pass of the headline.
set -e
export TMPDIR=/tmp
O=gpurun_out/prof2
mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4"
C="python3 bench.py --only-c4 --steps 2 --no-timing --c4-batch 16"
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c4b16_fetch -- $C > $O/pmc_c4b16_fetch.log 2>&1
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_c4b16_write -- $C > $O/pmc_c4b16_write.log 2>&1
SUTA_BF16_PLANES=0 timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c4np_fetch -- $C > $O/pmc_c4np_fetch.log 2>&1
SUTA_BF16_PLANES=0 timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_c4np_write -- $C > $O/pmc_c4np_write.log 2>&1
timeout -s KILL 170 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_sq -- $B > $O/pmc_sq.log 2>&1
echo done
