# Kernel trace of one rank's replayed row slab (tools/rank_sim.py --mode rows) for timeline
# analysis.  Usage on the box: bash tools/gpu_rowtrace.sh WORLD
set -e
export TMPDIR=/tmp
O=gpurun_out/rowtrace; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/rank_sim.py --mode rows --world ${1:-8} --rank 0 > $O/sim.json 2> $O/sim.err
