# Full round check on the GPU box: parity tests, smoke, bench, rocprof kernel-trace stats.
set -e
export TMPDIR=/tmp
O=gpurun_out/full
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err
