# Lag-Gram kernel tests, then grid A/B of the chain/gradient co-residency knobs
set -e
export TMPDIR=/tmp
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "lag_gram or first_gram" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 500 python -u tools/grid_ab.py 6 base: nococh:XTR_COCHAIN=False split1:CHOL_SPLIT=1 nolag:LAG_GRAM=False > $O/ab.json 2> $O/ab.err
