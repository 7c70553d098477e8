# C2 GEMM traffic with the band tile order (SUTA_GEMM_ORDER=8) vs the default, per GEMM grid.
set -e
export TMPDIR=/tmp
O=gpurun_out/r3ord
R=/tmp/r3ord_raw
mkdir -p $O $R
B="python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4"
csv() { find $R/$1 -name "*counter_collection.csv" | head -1; }
for g in 8 4; do
SUTA_GEMM_ORDER=$g timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/f$g -- $B > $O/f$g.log 2>&1
SUTA_GEMM_ORDER=$g timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/w$g -- $B > $O/w$g.log 2>&1
python3 tools/pmc_traffic.py $(csv f$g) $(csv w$g) $O/pmc_traffic_order$g.json > $O/pmc_traffic_order$g.txt
python3 tools/pmc_traffic.py $(csv f$g) $(csv w$g) --by-grid > $O/pmc_traffic_order${g}_by_grid.txt
rm -rf $R/*
done
echo done
