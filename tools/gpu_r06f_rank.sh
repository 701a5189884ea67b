# Simulated per-rank shares of the C4 grid at 2 / 4 / 8 ranks, median of 3 timed runs per rank.
set -e
O=gpurun_out/${1:-p6f}; mkdir -p $O
for w in 2 4 8; do timeout -k 10 300 python3 tools/rank_sim.py --world $w --all > $O/rank_$w.json 2> $O/rank_$w.err; done
echo done
