# bitwise GEMM-form tests, then C4 kernel traces: the remap library (tools/ab/libsuta_remap.so) against the in-tree one
set -e
export TMPDIR=/tmp
O=gpurun_out/r6${1:-nat}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large_bf16.py -k "hbx or conv_input or fused_delta or tn_form" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/r6/gpu_trace_ab.sh ${1:-nat} SUTA_LIB=$PWD/tools/ab/libsuta_remap.so -
