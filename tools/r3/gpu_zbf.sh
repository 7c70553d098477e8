# bf16 storage of the conv stack's z_i / da_i (SUTA_CONV_Z_BF16) + branch-free GELU in the fp32 paths: full GPU suite,
# smoke, default bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3zbf
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rA --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
echo done
