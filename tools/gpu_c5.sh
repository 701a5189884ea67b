# C5 (multi-response elastic-net path): the bench line, a kernel trace of the same command, and
# the HBM fetch of its kernels (FETCH_SIZE pass) -- which of Gram / X^T y / CD bounds the step.
set -e
export TMPDIR=/tmp
O=gpurun_out/c5; mkdir -p $O
timeout -k 10 300 python bench.py --config c5 --steps 2 --warmup 1 --no-cpu > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu > $O/bench_c5_kt.json 2> $O/kt.err
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu > $O/fetch.log 2>&1
