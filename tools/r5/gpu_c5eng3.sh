# C5 with 2 / 3 / 4 engines sharing the ragged groups, same box
set -e
export TMPDIR=/tmp
O=gpurun_out/r5c5eng3
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for e in 2 3 4 2 3; do
  timeout -k 10 300 python bench.py --only-c5 --no-timing --c5-engines $e > $O/c5_e$e.json 2> $O/c5_e$e.err
  python -c "import json; d=json.load(open('$O/c5_e$e.json')); print('C5 engines=$e', d['value'], d['audio_s_per_s'])"
done
