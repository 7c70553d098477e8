set -e
export TMPDIR=/tmp
O=gpurun_out/r2p
mkdir -p $O
timeout -k 10 120 ./tools/hb_bench 20 > $O/hb.log 2>&1
echo done
