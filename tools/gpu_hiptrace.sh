# Kernel + HIP API trace of C4 grids (tools/grid_ab.py, variant $1): host launch timing
set -e
export TMPDIR=/tmp
O=gpurun_out/ht; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/kt -o run -- python3 tools/grid_ab.py 2 "$1" > $O/ab.json 2> $O/ab.err
