# fp32 flash after a change: attn_bench (C2 shape x2, ragged edge shapes) and the fp32 attention parity tests.  $1 = tag
set -e
export TMPDIR=/tmp
O=gpurun_out/r6${1:-fp32attn}
mkdir -p $O
for r in 1 2; do timeout -k 10 120 ./tools/attn_bench 0 164 399 12 10 >> $O/ab.txt 2>&1; done
for T in 262 49 1874; do timeout -k 10 120 ./tools/attn_bench 0 24 $T 12 3 >> $O/ab.txt 2>&1; done
cat $O/ab.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "fused_attention or base_forward or longest or shortest or base_suta" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
