# Cholesky look-ahead: kernel test at depth 3 (ragged groups) and 4, then suite, bench, 8-rank sim,
# single-group kernel trace.
set -e
export TMPDIR=/tmp
O=gpurun_out/ck6; mkdir -p $O
SGLM_CHOL_LOOKAHEAD=3 timeout -k 10 200 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "chol" --timeout 120 --timeout-method thread > $O/la3.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 > $O/bench.json 2> $O/bench.err
SGLM_CHOL_LOOKAHEAD=2 timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 1 > $O/bench_la2.json 2> $O/bench_la2.err
timeout -k 10 300 python tools/rank_sim.py --world 8 --all > $O/all8.log 2>&1
SGLM_CHOL_LOOKAHEAD=2 timeout -k 10 300 python tools/rank_sim.py --world 8 --all > $O/all8_la2.log 2>&1
SGLM_IRLS_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/b.json 2> $O/b.err
