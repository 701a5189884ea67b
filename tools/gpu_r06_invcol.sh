# Round-6: the inverse by left-looking block columns beside the factorisation (SGLM_INV_COL)
# -- chol kernel tests, the chain alone at 1 / 3 / 11 / 20 representatives, the C4 grid A/B.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-invcol}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -k "chol" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python3 -u tools/chol_bench.py --n 1 3 11 20 --env SGLM_INV_COL=1,0 > $O/chain.json 2> $O/chain.err
timeout -k 10 400 python3 -u tools/grid_ab.py 6 col:env.SGLM_INV_COL=1 lev:env.SGLM_INV_COL=0 > $O/ab.json 2> $O/ab.err
echo done
