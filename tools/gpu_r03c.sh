# Gradient kernel variants: parity tests of the kernel path, then grid A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 500 python -u tools/grid_ab.py 6 base: nowpe2:env.SGLM_XTR_WPE2=0 > $O/ab.json 2> $O/ab.err
