# Lag-gradient check: kernel test, API + full-size parity, bench A/B (lag vs bit-plane MFMA).
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-lag}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "lag_xtr" tests/test_gpu_api.py tests/test_gpu_fullsize.py -k "lag_xtr or c3 or reuse or c2 or c4_grid or newton" -s > $O/tests.log 2>&1
SGLM_LAG_XTR=1 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_lag.json 2> $O/bench_lag.err
SGLM_LAG_XTR=0 timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_bits.json 2> $O/bench_bits.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/kt_bench.json 2> $O/kt.err
