# Round-6b: the stopping tolerance (STOP_TOL) against the grid's Newton iterations and time,
# then the full-size parity test (every fit's float64 Newton distance <= 1e-5) at 3e-6
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-stoptol}; mkdir -p $O
timeout -k 10 700 python3 -u tools/grid_ab.py 8 base: t3:STOP_TOL=3e-6 t10:STOP_TOL=1e-5 > $O/ab.json 2> $O/ab.err
SGLM_STOP_TOL=3e-6 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v -k "newton_distance or oracle" --timeout 500 --timeout-method thread > $O/full3.log 2>&1
echo done
