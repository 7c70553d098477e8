# Closing bench line on HEAD (default flags: 164 utterances, C2 + split + C4 + CPU baseline, PMC traffic from the
# closing passes) and smoke.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3final
mkdir -p $O
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err
echo done
