# Development check on the box: GPU parity suite, the default bench line, a kernel trace of
# the bench and an 8-rank share simulation.  Usage: bash tools/gpu_check.sh [pytest args]
set -e
export TMPDIR=/tmp
O=gpurun_out/chk; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread "$@" > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_g1.json 2> $O/kt1.err
timeout -k 10 300 python -u tools/rank_sim.py --world 8 --all > $O/rank8.json 2> $O/rank8.err
