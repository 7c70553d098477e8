set -e
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -- python3 bench.py --steps 2 --warmup 1 --no-split --no-cpu-baseline --no-timing --no-c4 > $O/kt.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c4 -- python3 bench.py --only-c4 --steps 2 --no-timing > $O/kt_c4.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -- python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4 > $O/pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -- python3 bench.py --steps 1 --warmup 0 --no-split --no-cpu-baseline --no-timing --no-c4 > $O/pmc_write.log 2>&1
echo done
