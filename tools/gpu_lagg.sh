# Lag-Gram tests and its kernel time inside the C4 grid (kernel-trace stats)
set -e
export TMPDIR=/tmp
O=gpurun_out/lagg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "lag_gram or first_gram" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/grid_ab.py 2 base: > $O/ab.json 2> $O/ab.err
