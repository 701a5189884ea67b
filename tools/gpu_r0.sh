set -e
O=gpurun_out/r0; mkdir -p $O
SIM_WARMUPS=2 timeout -k 10 300 python tools/rank_sim.py --world 8 --rank 4 > $O/r4w2.log 2>&1
SIM_WARMUPS=3 timeout -k 10 300 python tools/rank_sim.py --world 8 --rank 4 > $O/r4w3.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --steps 4 --warmup 1 > $O/b.json 2>&1
