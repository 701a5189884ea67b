# Round artifacts: PMC traffic of the Gram (separate FETCH/WRITE passes), the default bench line
# (with CPU baseline), and the rocprofv3 kernel-trace summary of the same bench command.
set -e
export TMPDIR=/tmp
O=gpurun_out/prof; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/write.log 2>&1
python tools/pmc_traffic.py $O/fetch $O/write profiles/r01_pmc_traffic.json > $O/pmc.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/kt.err
timeout -k 10 400 python bench.py --config c5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
