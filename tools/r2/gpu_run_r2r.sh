set -e
export TMPDIR=/tmp
O=gpurun_out/r2r
mkdir -p $O
C="python3 bench.py --only-c4 --steps 2 --no-timing"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -- $C > $O/kt_c4.log 2>&1
echo done
