# Kernel trace of the default bench (2 timed grids) for timeline analysis (tools/timeline.py).
set -e
export TMPDIR=/tmp
O=gpurun_out/t4; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-dropin > $O/bench.json 2> $O/bench.err
