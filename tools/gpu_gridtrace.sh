# Kernel trace of C4 grids run by tools/grid_ab.py (variant given as $1), for timeline analysis
set -e
export TMPDIR=/tmp
O=gpurun_out/gt; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/grid_ab.py 2 "$1" > $O/ab.json 2> $O/ab.err
