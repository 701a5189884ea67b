# Knob sweep on the C4 bench (tolerances, IRLS groups) and simulated rank shares.
set -e
export TMPDIR=/tmp
O=gpurun_out/sw; mkdir -p $O
run() { timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_$1.json 2> $O/bench_$1.err; }
run base
SGLM_IRLS_GROUPS=1 run g1
SGLM_HESS_SHARE_TOL=0.75 run share075
SGLM_HESS_SHARE_TOL=0.75 SGLM_HESS_REUSE_TOL=0.75 run both075
SGLM_HESS_SHARE_TOL=0.75 SGLM_HESS_REUSE_TOL=0.5 SGLM_IRLS_GROUPS=1 run s075r05g1
timeout -k 10 300 python -u tools/rank_sim.py --world 8 --all > $O/rank8.json 2> $O/rank8.err
timeout -k 10 300 python -u tools/rank_sim.py --world 2 --all > $O/rank2.json 2> $O/rank2.err
