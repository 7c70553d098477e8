# C4 kernel traces of several library / environment configurations (one bench call each, eager): $1 = output tag,
# then one argument per configuration ("-" = defaults, else space-separated VAR=value pairs, e.g. SUTA_LIB=...)
set -e
export TMPDIR=/tmp
export SUTA_GRAPHS=0
O=gpurun_out/r6$1
mkdir -p $O
shift
i=0
for c in "$@"; do
  i=$((i+1))
  if [ "$c" = "-" ]; then c=""; fi
  R=/tmp/trab_$i
  env $c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R -- python3 bench.py --only-c4 --steps 1 --warmup 0 --no-timing > $O/kt$i.log 2>&1
  echo "[$c]" > $O/trace$i.txt
  python3 tools/trace_summary.py $(find $R -name "*kernel_trace.csv" | head -1) >> $O/trace$i.txt
  rm -rf $R
  echo "config $i done"
done
