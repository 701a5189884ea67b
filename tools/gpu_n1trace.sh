set -e
export TMPDIR=/tmp
O=gpurun_out/n1t; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/b.json 2> $O/b.err
