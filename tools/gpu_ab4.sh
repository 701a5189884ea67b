# Round-4 kernel variants: their equality tests, the gradient micro A/B, the C4 grid A/B of the
# pipelined gradient and the XCD-banded Gram, then the C5 profile (tools/gpu_c5.sh).
set -e
export TMPDIR=/tmp
O=gpurun_out/ab4; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "xtr or xcd" > $O/kern_tests.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_api.py -k "enet" > $O/enet_tests.log 2>&1
timeout -k 10 200 python -u tools/ab_micro.py xtr 120,70 > $O/ab_xtr.log 2>&1
timeout -k 10 400 python -u tools/grid_ab.py 6 base: pipe:env.SGLM_XTR_PIPE=1 xcd:env.SGLM_SYRK_XCD=1 both:env.SGLM_XTR_PIPE=1,env.SGLM_SYRK_XCD=1 > $O/grid_ab.log 2>&1
bash tools/gpu_c5.sh
