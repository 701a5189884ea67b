# Round-6b: worst float64 Newton distance over the C4 grid's 120 fits at STOP_TOL 1e-6 / 3e-6 /
# 1e-5 (tests/test_gpu_fullsize.py prints it; -s)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-stoptol2}; mkdir -p $O
for t in 1e-5 3e-6 1e-6; do
SGLM_STOP_TOL=$t timeout -k 10 400 python3 -u -m pytest tests/test_gpu_fullsize.py -x -s -q -k "newton_distance_float64_every_fit or converges" --timeout 350 --timeout-method thread > $O/full_$t.log 2>&1
done
echo done
