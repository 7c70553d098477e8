# C5 at the 512-utterance sample: --c5-gpu-min-fill sweep (same box, two rounds); $1 = tag, MFS = values
set -e
export TMPDIR=/tmp
O=gpurun_out/r5c5_${1:-mf}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for i in 1 2; do
  for mf in ${MFS:-0.2 0.4 0.7}; do
    timeout -k 10 300 python bench.py --only-c5 --c5-gpu-min-fill $mf > $O/c5_mf$mf.$i.json 2> $O/c5_mf$mf.$i.err
    python -c "import json; d=json.load(open('$O/c5_mf$mf.$i.json')); print('C5 mf=$mf', d['value'], d['audio_s_per_s'], d['padded_frame_fraction'], d['n_batches'], d['roofline']['frac'])"
  done
done
