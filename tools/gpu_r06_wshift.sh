# Round-6b: structured Gram with each piece's column window at its first d row
# (SGLM_LAGW_WSHIFT) and the first iteration's link + gradient once per start key (GRAD_DEDUP)
# -- the structured-Gram, mixed, f32-design and API tests, the standalone Gram A/B (H bitwise
# with the split off) and the C4 grid A/B.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-wsh}; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_laggram_w.py tests/test_gpu_mixed_structured.py tests/test_gpu_f32design.py tests/test_gpu_api.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
LAGW_ENV=SGLM_LAGW_WSHIFT=1,0 timeout -k 10 300 python3 -u tools/lagw_bench.py > $O/lagw.json 2> $O/lagw.err
timeout -k 10 500 python3 -u tools/grid_ab.py 6 base: v3:env.SGLM_LAGW_WSHIFT=0 nodedup:GRAD_DEDUP=False > $O/ab.json 2> $O/ab.err
echo done
