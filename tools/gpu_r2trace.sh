set -e
export TMPDIR=/tmp
O=gpurun_out/r2t; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/rank_sim.py --world 8 --rank 2 > $O/r2.log 2>&1
