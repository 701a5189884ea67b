set -e
mkdir -p gpurun_out/q
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/q/tests.log 2>&1
timeout -k 10 200 python tools/bench_kernels.py --variants 6 --fits 120 --reps 3 --other > gpurun_out/q/k120.log 2>&1
timeout -k 10 200 python tools/bench_kernels.py --variants 6 --fits 15 --reps 3 --other > gpurun_out/q/k15.log 2>&1
timeout -k 10 400 python tools/rank_sim.py --world 8 --rank 5 > gpurun_out/q/r5of8.log 2>&1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/q/b.log 2>&1
