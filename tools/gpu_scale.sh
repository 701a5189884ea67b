set -e
O=gpurun_out/scale; mkdir -p $O
for w in 2 4 8; do timeout -k 10 300 python tools/rank_sim.py --world $w --all > $O/w$w.log 2>&1; done
timeout -k 10 300 python bench.py --no-cpu --steps 4 --warmup 1 > $O/b1.json 2>/dev/null
