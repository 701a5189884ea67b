# Round-6: structured Gram piece order -- XCD-local ranges (default) vs longest-piece-first
# (SGLM_LAGW_ORDER=1): correctness, standalone timing, C4 grids interleaved.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-ord}; mkdir -p $O
timeout -k 10 300 env SGLM_LAGW_ORDER=1 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_laggram_w.py > $O/tests_lpt.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_xcd.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LAGW_ORDER=1 python3 tools/lagw_bench.py > $O/time_lpt.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_xcd.json 2> $O/bench_xcd.err
timeout -k 10 300 env SGLM_LAGW_ORDER=1 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_lpt.json 2> $O/bench_lpt.err
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_xcd2.json 2> $O/bench_xcd2.err
timeout -k 10 300 env SGLM_LAGW_ORDER=1 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_lpt2.json 2> $O/bench_lpt2.err
echo done
