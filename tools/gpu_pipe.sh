# Gram/chain pipelining: parity tests that exercise the grid, the C4 bench A/B (same box,
# alternating), a kernel trace of the default.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-pipe}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_fullsize.py tests/test_gpu_api.py > $O/tests.log 2>&1
for v in 2 0 2 0 2 0; do
  SGLM_GRAM_PIPE=$v timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu >> $O/bench_$v.json 2>> $O/bench_$v.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/kt.json 2> $O/kt.err
