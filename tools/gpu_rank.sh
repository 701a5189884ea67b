# One simulated rank share of an 8-GPU C4 grid: phases and a kernel trace.
set -e
export TMPDIR=/tmp
O=gpurun_out/rank; mkdir -p $O
timeout -k 10 300 python3 -u tools/rank_sim.py --world 8 --rank 0 > $O/rank1.json 2> $O/rank1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/rank_sim.py --world 8 --rank 0 > $O/rank1_prof.json 2> $O/kt.err
