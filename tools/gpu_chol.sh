# Factorisation-chain experiment on the box: the GPU suite, the chain timing with the single-
# and four-wave diagonal steps, a kernel trace of the chain, an 8-rank share with phases and the
# default bench line.   Usage: bash tools/gpu_chol.sh [pytest -k expression]
set -e
export TMPDIR=/tmp
O=gpurun_out/chol; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${1:+-k "$1"} > $O/tests.log 2>&1
SGLM_DIAG4=0 timeout -k 10 120 python -u tools/chol_bench.py > $O/chain_d1.json 2> $O/chain_d1.err
timeout -k 10 120 python -u tools/chol_bench.py > $O/chain_d4.json 2> $O/chain_d4.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/chol_bench.py --n 3 --reps 10 > $O/chain_prof.json 2> $O/kt.err
timeout -k 10 300 python -u tools/rank_sim.py --world 8 --rank 2 > $O/rank8_r2.json 2> $O/rank8_r2.err
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench.json 2> $O/bench.err
SGLM_CHOL_STREAM=prio timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_prio.json 2> $O/bench_prio.err
