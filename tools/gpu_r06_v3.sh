# Round-6: structured Gram v3 staging (buffer loads with range-checked zeros, per-occurrence
# addresses computed once, exact task counts per half count) and split heavy pieces -- parity
# tests, standalone timing against the previous library, C4 grids interleaved.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-v3}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_laggram_w.py tests/test_gpu_mixed_structured.py > $O/tests.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_new.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LAGW_SPLIT=0 python3 tools/lagw_bench.py > $O/time_nosplit.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LIB=$V/libsglm_prev.so python3 tools/lagw_bench.py > $O/time_prev.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_new.json 2> $O/bench_new.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_prev.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_prev.json 2> $O/bench_prev.err
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_new2.json 2> $O/bench_new2.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_prev.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_prev2.json 2> $O/bench_prev2.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-dropin --no-check > $O/bench_prof.json 2> $O/kt.err
echo done
