# Round-6b: split-precision (bf16 x3) inversion levels (SGLM_INV_X3) -- the chol kernel tests
# with it on, the chain alone A/B, the C4 grid A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-x3}; mkdir -p $O
SGLM_INV_X3=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -k "chol and not equal_levels and not four_pivots" --timeout 120 --timeout-method thread > $O/chol.log 2>&1
timeout -k 10 300 python3 -u tools/chol_bench.py --n 1 6 11 20 --env SGLM_INV_X3=1,0 > $O/chain.json 2> $O/chain.err
timeout -k 10 500 python3 -u tools/grid_ab.py 8 base: x3:env.SGLM_INV_X3=1 > $O/ab.json 2> $O/ab.err
echo done
