# Sweep the Hessian reuse / sharing tolerances over the C4 bench (development tool).
set -e
O=gpurun_out/tol5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for rs in "0.375 0.375" "0.5 0.5" "0.25 0.25"; do
  set -- $rs
  SGLM_HESS_REUSE_TOL=$1 SGLM_HESS_SHARE_TOL=$2 timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > $O/b_$1_$2.json 2> /dev/null
done
SGLM_HESS_REUSE_TOL=0.5 SGLM_HESS_SHARE_TOL=0.5 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests05.log 2>&1
