# Gradient row-slab choice: kernel tests, micro-benchmark at several fit counts, C4 bench.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-xtrsplit}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k xtr > $O/k.log 2>&1
SGLM_XTR4=1 timeout -k 10 200 python -u tools/lag_bench.py 120,96,70,40,16,6 bits > $O/micro4.log 2>&1
SGLM_XTR4=0 timeout -k 10 200 python -u tools/lag_bench.py 120,96,70,40,16,6 bits > $O/micro1.log 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench.json 2> $O/bench.err
