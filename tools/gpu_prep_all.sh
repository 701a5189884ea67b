# Session preprocessing: GPU parity tests, then the bench line and its kernel-trace summary.
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/prep
timeout -k 10 300 python -u -m pytest tests/test_gpu_prep.py -x -v --timeout 120 --timeout-method thread > gpurun_out/prep/tests.log 2>&1
bash tools/gpu_prep_bench.sh
