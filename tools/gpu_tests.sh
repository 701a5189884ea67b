# GPU parity suite (optionally a subset: extra pytest args), then one default bench line.
# Usage on the box: bash tools/gpu_tests.sh [pytest args...]
set -e
export TMPDIR=/tmp
O=gpurun_out/tests; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread "$@" > $O/tests.log 2>&1
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
