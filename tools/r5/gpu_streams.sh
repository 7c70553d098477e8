# Several engines per GPU (tools/bench_streams.py) at the bench batch: C4 and C2, 2 engines x 82 utterances vs 1 x 164
set -e
export TMPDIR=/tmp
O=gpurun_out/r5streams
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python tools/bench_streams.py --c4 --engines 2 --batch 164 --warmup 2 --steps 3 > $O/c4_e2.json 2> $O/c4_e2.err
cat $O/c4_e2.json
timeout -k 10 400 python tools/bench_streams.py --engines 2 --batch 164 --warmup 2 --steps 3 > $O/c2_e2.json 2> $O/c2_e2.err
cat $O/c2_e2.json
