# Same-box A/B: config C4 over variants given as "NAME=VAL[,NAME=VAL]" (or "base"), config C2 (headline line only) over
# SUTA_FLASH_FWD_PIPE; interleaved rounds; $1 = output tag, C4VARS / C2VARS override the variant lists
set -e
export TMPDIR=/tmp
O=gpurun_out/r5ab_${1:-ab}
mkdir -p $O
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
[ -n "$PRETEST" ] && { timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread $PRETEST > $O/pretest.log 2>&1 || { tail -40 $O/pretest.log; exit 1; }; tail -1 $O/pretest.log; }
C4VARS=${C4VARS:-"base SUTA_HBX_FORM=2 SUTA_HBP_CONV=0 SUTA_HBX_FORM=2,SUTA_HBP_CONV=0"}
C2VARS=${C2VARS:-"base SUTA_FLASH_FWD_PIPE=0"}
run() {  # $1 variant, $2 round, $3 c2|c4
  local envs=""
  [ "$1" != base ] && envs=$(echo $1 | tr ',' ' ')
  local tag=$(echo $1 | tr ',=' '_-')
  if [ $3 = c4 ]; then
    env $envs timeout -k 10 300 python bench.py --only-c4 --steps 4 > $O/c4_$tag.$2.json 2> $O/c4_$tag.$2.err
    python -c "import json; d=json.load(open('$O/c4_$tag.$2.json')); print('C4 $1', d['value'], d['roofline']['frac'], 'attn', d['attention']['tflops'], d['time_breakdown_ms'])"
  else
    env $envs timeout -k 10 300 python bench.py --no-c4 --no-c5 --no-batch64 --no-split --no-cpu-baseline --steps 4 > $O/c2_$tag.$2.json 2> $O/c2_$tag.$2.err
    python -c "import json; d=json.load(open('$O/c2_$tag.$2.json')); print('C2 $1', d['value'], d['roofline']['frac'], 'attn', d['attention']['tflops'], d.get('time_breakdown_ms'))"
  fi
}
for i in 1 2; do
  for v in $C4VARS; do run $v $i c4; done
  for v in $C2VARS; do run $v $i c2; done
done
