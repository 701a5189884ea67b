# Round-4 checks after the pipelined-gradient default and the C5 scoring rewrite.
set -e
export TMPDIR=/tmp
O=gpurun_out/ab5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "xtr" > $O/kern_tests.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_api.py -k "enet" > $O/enet_tests.log 2>&1
timeout -k 10 200 python -u tools/ab_micro.py xtrd 120,70,40 > $O/ab_xtrd.log 2>&1
timeout -k 10 400 python -u tools/grid_ab.py 6 base: pipe0:env.SGLM_XTR_PIPE=0 > $O/grid_ab.log 2>&1
bash tools/gpu_c5.sh
