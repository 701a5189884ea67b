# GPU suite, the upload A/B and the Hessian-reuse tolerance sweep at the 8-rank share and on
# one GPU (after the chain speed-ups the balance between a fresh Hessian and an extra Newton
# iteration moved).   Usage: bash tools/gpu_tol.sh
set -e
export TMPDIR=/tmp
O=gpurun_out/tol; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_up_$rep.json 2> $O/bench_up_$rep.err
  SGLM_UPLOAD_TORCH=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_torch_$rep.json 2> $O/bench_torch_$rep.err
done
SGLM_UPLOAD_TORCH=1 timeout -k 10 300 python -u tools/rank_sim.py --world 8 --all > $O/rank8_torch.json 2> $O/rank8_torch.err
for t in 0.375 0.5 0.75 1.0; do
  SGLM_HESS_REUSE_TOL=$t timeout -k 10 300 python -u tools/rank_sim.py --world 8 --all > $O/rank8_$t.json 2> $O/rank8_$t.err
  SGLM_HESS_REUSE_TOL=$t timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_$t.json 2> $O/bench_$t.err
done
