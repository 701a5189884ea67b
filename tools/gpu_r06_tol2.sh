# Round-6b: lower Hessian-reuse / cross-mask tolerances (more fresh Hessians, fewer tail iterations?)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-tol2}; mkdir -p $O
timeout -k 10 700 python3 -u tools/grid_ab.py 8 base: r025:HESS_REUSE_TOL=0.25 x05:HESS_XMASK_TOL=0.5 x1:HESS_XMASK_TOL=1.0 s025:HESS_SHARE_TOL=0.25 > $O/ab.json 2> $O/ab.err
echo done
