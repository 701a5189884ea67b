# Round-6b: inverses formed after the solve (sglm_chol_factor / sglm_chol_invert, the fresh
# factors solved by substitution) -- chol tests, the full-size parity suite, the C4 grid A/B.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-defer}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_kernels.py -x -q -k "chol" --timeout 120 --timeout-method thread > $O/chol.log 2>&1
timeout -k 10 600 python3 -u tools/grid_ab.py 8 base: nodefer:DEFER_INV_MIN=0 d6:DEFER_INV_MIN=6 > $O/ab.json 2> $O/ab.err
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_api.py -x -v --timeout 600 --timeout-method thread > $O/full.log 2>&1
echo done
