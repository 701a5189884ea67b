# Direction-product kernel: kernel tests, C4 bench with the staged kernel on and off, kernel stats.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-eta}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "eta" > $O/k.log 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_on.json 2> $O/bench_on.err
SGLM_ETA_DIR=0 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_off.json 2> $O/bench_off.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/kt.json 2> $O/kt.err
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "xtr" > $O/kx.log 2>&1
timeout -k 10 200 python -u tools/lag_bench.py 120,96,70,40,16,6 bits > $O/micro_g2.log 2>&1
SGLM_XTR_NGW=1 timeout -k 10 200 python -u tools/lag_bench.py 120,96,70,40,16,6 bits > $O/micro_g1.log 2>&1
