# Session-preprocessing bench line + rocprofv3 kernel-trace summary of the same command.
set -e
export TMPDIR=/tmp
O=gpurun_out/prepb; mkdir -p $O
timeout -k 10 300 python bench.py --config prep --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --config prep --steps 5 --warmup 2 --no-cpu > $O/bench_prof.json 2> $O/kt.err
