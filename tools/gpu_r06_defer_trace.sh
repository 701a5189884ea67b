# Round-6b: kernel trace of C4 grids with the deferred inversion on (timeline of its solves)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-dtr}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/grid_ab.py 2 d:DEFER_INV_MIN=10 > $O/ab.json 2> $O/ab.err
echo done
