# Four-panel gradient kernel: its test, the micro-benchmark against the one-panel kernel, and
# the C4 bench A/B (also the stopping tolerance 1e-6 vs 4e-6).
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-xtr4}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 -p no:cacheprovider tests/test_gpu_kernels.py -k "xtr" > $O/tests.log 2>&1
SGLM_XTR4=1 timeout -k 10 200 python -u tools/lag_bench.py 120,16,6 bits > $O/micro4.log 2>&1
SGLM_XTR4=0 timeout -k 10 200 python -u tools/lag_bench.py 120,16,6 bits > $O/micro1.log 2>&1
for v in x4 x1 x4tol; do
  case $v in x4) export SGLM_XTR4=1 SGLM_STOP_TOL=1e-6;; x1) export SGLM_XTR4=0 SGLM_STOP_TOL=1e-6;; x4tol) export SGLM_XTR4=1 SGLM_STOP_TOL=4e-6;; esac
  timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err
done
