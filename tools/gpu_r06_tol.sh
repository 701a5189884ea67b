# Round-6b: the first-iteration gradient dedup and the Hessian-reuse / sharing tolerances at the
# 30 ms grid (one process, alternating grids), then a kernel trace of the default grid.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-tol}; mkdir -p $O
timeout -k 10 700 python3 -u tools/grid_ab.py 10 base: nodedup:GRAD_DEDUP=False r05:HESS_REUSE_TOL=0.5 r075:HESS_REUSE_TOL=0.75 s05:HESS_SHARE_TOL=0.5 > $O/ab.json 2> $O/ab.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/grid_ab.py 2 base: > $O/kt_ab.json 2> $O/kt.err
echo done
