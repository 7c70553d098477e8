# Round-5 HBM traffic evidence at the bench defaults: rocprofv3 FETCH_SIZE and WRITE_SIZE passes (separate runs, as
# MI355X_MICROARCH.md prescribes) of one workload ($1 = c2 | c4), reduced per kernel family and per GEMM grid by
# tools/pmc_traffic.py into gpurun_out/r5prof/pmc_traffic{,_c4}.json (bench.py reads the newest committed round's)
set -e
( while sleep 50; do echo "tick $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
export SUTA_GRAPHS=0   # rocprofv3 --pmc crashes on a launched hipGraph; eager runs the same kernels
w=$1
O=gpurun_out/r5prof
R=/tmp/r5traffic_raw_$w
mkdir -p $O $R
if [ $w = c2 ]; then X="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4 --no-c5 --no-batch64"; S=""
else X="python3 bench.py --only-c4 --steps 1 --warmup 0 --no-timing"; S="_c4"; fi
csv() { find $R/$1 -name "*counter_collection.csv" | head -1; }
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -- $X > $O/${w}_fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -- $X > $O/${w}_write.log 2>&1
python3 tools/pmc_traffic.py $(csv fetch) $(csv write) $O/pmc_traffic$S.json > $O/pmc_traffic$S.txt
python3 tools/pmc_traffic.py $(csv fetch) $(csv write) --by-grid > $O/pmc_traffic${S}_by_grid.txt
rm -rf $R
echo done
