# Complement first Grams: their tests, the C4 grid A/B (on / off), one bench line.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab6; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "complement or first_gram" > $O/tests.log 2>&1
timeout -k 10 400 python -u tools/grid_ab.py 6 base: nocomp:COMP_GRAM=False > $O/grid_ab.log 2>&1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu > $O/bench.json 2> $O/bench.err
