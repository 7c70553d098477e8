set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r6nat
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_large_bf16.py -k "hbx or conv_input or fused_delta" > gpurun_out/r6nat/tests.log 2>&1 || { tail -40 gpurun_out/r6nat/tests.log; exit 1; }
tail -1 gpurun_out/r6nat/tests.log
bash tools/r6/gpu_trace_ab.sh nat SUTA_LIB=$PWD/tools/ab/libsuta_remap.so -
