set -e
O=gpurun_out/rep; mkdir -p $O
for i in 1 2 3; do timeout -k 10 300 python bench.py --no-cpu --steps 4 --warmup 1 > $O/b$i.json 2>/dev/null; done
for i in 1 2; do timeout -k 10 300 python tools/rank_sim.py --world 8 --all > $O/a$i.log 2>&1; done
