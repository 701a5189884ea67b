# Kernel traces (per-dispatch CSV) of the C4 bench grid and the designmat bench, for timeline
# analysis (tools/timeline.py).  Usage on the box: bash tools/gpu_trace.sh OUTDIR
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-trace}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/c4_bench.json 2> $O/c4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dm -o run -- python3 bench.py --config designmat --steps 3 --warmup 1 --no-cpu > $O/dm_bench.json 2> $O/dm.err
