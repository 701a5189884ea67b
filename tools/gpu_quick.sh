set -e
mkdir -p gpurun_out/ab
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q > gpurun_out/ab/tests.log 2>&1
timeout -k 10 200 python tools/bench_kernels.py --variants 6 --masked --fits 120 --reps 5 > gpurun_out/ab/k.log 2>&1
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/ab/b.log 2>&1
