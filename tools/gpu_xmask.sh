# Cross-mask Hessian sharing: bench at several alias tolerances, then kernel traces at one.
# Usage on the box: bash tools/gpu_xmask.sh TOL_FOR_TRACE
set -e
export TMPDIR=/tmp
O=gpurun_out/xm2; mkdir -p $O
for t in 0.75 1.0 1.5 2.0; do
  SGLM_HESS_XMASK_TOL=$t timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_$t.json 2> $O/bench_$t.err
done
export SGLM_HESS_XMASK_TOL=${1:-1.0}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/kt.err
SGLM_IRLS_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_prof_g1.json 2> $O/kt1.err
SGLM_IRLS_GROUPS=1 timeout -k 10 200 python tools/grid_phases.py > $O/phases_g1.json 2> $O/phases.err
