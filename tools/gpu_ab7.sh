# Forked trailing updates in the factorisation chain: bitwise test, C4 grid A/B, chain micro.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab7; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "chol" > $O/tests.log 2>&1
timeout -k 10 500 python -u tools/grid_ab.py 8 fork:env.SGLM_CHOL_FORK=1 nofork:env.SGLM_CHOL_FORK=0 > $O/grid_ab.log 2>&1
