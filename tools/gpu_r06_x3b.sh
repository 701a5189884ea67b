# Round-6b: split-precision inversion levels on -- full-size parity + API suites, grid A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-x3b}; mkdir -p $O
timeout -k 10 600 python3 -u tools/grid_ab.py 10 base: x3:env.SGLM_INV_X3=1 > $O/ab.json 2> $O/ab.err
SGLM_INV_X3=1 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_api.py tests/test_gpu_api_rows.py tests/test_gpu_mixed_structured.py -x -v --timeout 600 --timeout-method thread > $O/full.log 2>&1
echo done
