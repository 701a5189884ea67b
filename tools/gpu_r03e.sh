# GPU suite at head + a short grid timing
set -e
export TMPDIR=/tmp
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 400 python -u tools/grid_ab.py 6 base: split2:CHOL_SPLIT=2 > $O/ab.json 2> $O/ab.err
