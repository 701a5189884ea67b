# Round-6b: narrow structured-Gram launches with four M tiles per wave (SGLM_LAGW_MT4)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-mt4}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_laggram_w.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
LAGW_ENV=SGLM_LAGW_MT4=1,0 timeout -k 10 300 python3 -u tools/lagw_bench.py > $O/lagw.json 2> $O/lagw.err
timeout -k 10 500 python3 -u tools/grid_ab.py 8 base: mt2:env.SGLM_LAGW_MT4=0 > $O/ab.json 2> $O/ab.err
echo done
