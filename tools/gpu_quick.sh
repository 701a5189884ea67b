# Quick development check on the box: kernel tests matching a pattern, the default bench line,
# an 8-rank share breakdown (phases of rank 1) and its kernel trace.
# Usage on the box: bash tools/gpu_quick.sh [pytest -k expression]
set -e
export TMPDIR=/tmp
O=gpurun_out/q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "${1:-chol}" > $O/tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -u tools/rank_sim.py --world 8 --rank 1 > $O/rank1.json 2> $O/rank1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/rank_sim.py --world 8 --rank 1 > $O/rank1_prof.json 2> $O/kt.err
