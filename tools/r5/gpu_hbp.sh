# hbp deep-prefetch form: bare-shape bench (tools/hb_bench), then the new GPU tests incl. the bitwise form test; $1 = tag
set -e
export TMPDIR=/tmp
O=gpurun_out/r5${1:-hbp}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 ./tools/hb_bench 10 3 > $O/hb_bench.log 2>&1 || { cat $O/hb_bench.log; exit 1; }
grep -E "hbx|hbp|epi" $O/hb_bench.log
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  "tests/test_gpu_large_bf16.py::test_bf16_hbx_slice_ring_kernel_bitwise_equals_128_tile" \
  "tests/test_gpu_large_bf16.py::test_conv_input_gradients_on_256_tile_bitwise" \
  "tests/test_gpu_parity.py::test_pipelined_fp32_flash_forward_bitwise" \
  "tests/test_gpu_parity.py::test_scheduler_and_sgd_match_reference" \
  "tests/test_gpu_parity.py::test_graph_replay_equals_eager" \
  "tests/test_gpu_large_bf16.py::test_batched_gemm_without_off32_epilogue_falls_back" \
  "tests/test_gpu_large_bf16.py::test_bf16_fused_delta_bitwise_equals_separate_pass" \
  "tests/test_gpu_cli.py::test_cli_scheduler_steplr" \
  "tests/test_gpu_bench_scale.py::test_bench_layout_matches_oracle" \
  "tests/test_gpu_bench_scale.py::test_c4_bench_layout_bf16" > $O/tests.log 2>&1 || { tail -80 $O/tests.log; exit 1; }
tail -3 $O/tests.log
