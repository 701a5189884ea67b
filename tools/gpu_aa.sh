# The secant (Anderson-1) direction correction: grid A/B, per-iteration log with it, and the
# full-size parity tests under it.  Usage on the box: bash tools/gpu_aa.sh
set -e
export TMPDIR=/tmp
O=gpurun_out/aa; mkdir -p $O
timeout -k 10 400 python -u tools/grid_ab.py 6 base:ANDERSON=False aa:ANDERSON=True > $O/ab.json 2> $O/ab.err
timeout -k 10 300 python -u tools/iter_log.py > $O/iterlog.txt 2> $O/iterlog.err
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_api.py tests/test_gpu_api_rows.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
