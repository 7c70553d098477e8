# Round-2 closing evidence on HEAD: GPU suite, smoke, bench line, kernel traces (headline, C4), C4 PMC passes.
set -e
export TMPDIR=/tmp
O=gpurun_out/prof2f
mkdir -p $O
for m in 0 3 4; do
SUTA_HB8=$m timeout -k 10 300 python bench.py --only-c4 --steps 2 --no-timing > $O/c4_hb8_$m.json 2> $O/c4_hb8_$m.err
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python3 bench.py --steps 2 --warmup 1 --no-split --no-cpu-baseline --no-timing --no-c4 > $O/kt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -- python3 bench.py --only-c4 --steps 2 --no-timing > $O/kt_c4.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c4_fetch -- python3 bench.py --only-c4 --steps 2 --no-timing > $O/pmc_c4_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_c4_write -- python3 bench.py --only-c4 --steps 2 --no-timing > $O/pmc_c4_write.log 2>&1
echo done
