set -e
export TMPDIR=/tmp
O=gpurun_out/r2v
mkdir -p $O
for i in 1 2; do
SUTA_QKV_PLANE=0 timeout -k 10 300 python bench.py --only-c4 --steps 2 --no-timing > $O/c4_off_$i.json 2> /dev/null
timeout -k 10 300 python bench.py --only-c4 --steps 2 --no-timing > $O/c4_on_$i.json 2> /dev/null
done
echo done
