# C5 with 1 / 2 engines (own streams and host threads) sharing the ragged groups; two rounds, same box
set -e
export TMPDIR=/tmp
O=gpurun_out/r5c5eng
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for i in ${ROUNDS:-1 2}; do
  for e in 1 2; do
    timeout -k 10 300 python bench.py --only-c5 --c5-engines $e > $O/c5_e$e.$i.json 2> $O/c5_e$e.$i.err
    python -c "import json; d=json.load(open('$O/c5_e$e.$i.json')); print('C5 engines=$e', d['value'], d['audio_s_per_s'], d['roofline']['frac'])"
  done
done
