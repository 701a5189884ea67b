# Round-4 check: the full GPU suite (stops at the first failure), then one default bench line.
# Usage on the box: bash tools/gpu_r04.sh [pytest args...]
set -e
export TMPDIR=/tmp
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread --durations=25 -p no:cacheprovider "$@" > $O/tests.log 2>&1
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
