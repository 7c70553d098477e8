# Config C5 grouping sweep: the driver's ragged_groups at several --gpu_min_fill values (bench.py --only-c5)
set -e
O=gpurun_out/r4c5
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for mf in ${MF:-0.35 0.2 0.1 0.05}; do
  timeout -k 10 300 python bench.py --only-c5 --c5-n ${N:-96} --c5-gpu-min-fill $mf > $O/c5_mf$mf.json 2> $O/c5_mf$mf.err
  python -c "import json,sys; d=json.load(open('$O/c5_mf$mf.json')); print('$mf', d['value'], d['audio_s_per_s'], d['padded_frame_fraction'], d['batch_sizes'], d['roofline']['frac'])"
done
