# Cross-mask Hessian sharing sweep: bench at several alias tolerances, then the parity suite.
set -e
export TMPDIR=/tmp
O=gpurun_out/xm; mkdir -p $O
for t in 0.5 0 1.0; do
  SGLM_HESS_XMASK_TOL=$t timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_$t.json 2> $O/bench_$t.err
done
SGLM_GROUP_SPLIT=snake timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_snake.json 2> $O/bench_snake.err
SGLM_IRLS_GROUPS=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_g1.json 2> $O/bench_g1.err
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 400 --timeout-method thread > $O/tests.log 2>&1
