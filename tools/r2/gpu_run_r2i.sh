set -e
export TMPDIR=/tmp
O=gpurun_out/r2i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_bf16.py -k "fused_attention or longest or bf16_large or planes" -x -q --timeout 200 --timeout-method thread > $O/attn.log 2>&1
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-split --no-c4 > $O/b.json 2>/dev/null
timeout -s KILL 170 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $O/pmc_sq -- python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4 > $O/pmc_sq.log 2>&1
echo done
