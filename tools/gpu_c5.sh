set -e
export TMPDIR=/tmp
O=gpurun_out/c5; mkdir -p $O
timeout -k 10 400 python bench.py --config c5 --steps 2 --warmup 1 > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > $O/prof.json 2> $O/prof.err
