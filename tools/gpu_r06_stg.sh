# Round-6: the structured Gram with the staging interleaved into the K-steps (default) against
# the previous head (staging after the barrier): correctness, standalone timing, C4 grid, PMC.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-stg}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_laggram_w.py > $O/tests.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_new.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LIB=$V/libsglm_prev.so python3 tools/lagw_bench.py > $O/time_prev.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_new.json 2> $O/bench_new.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_prev.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_prev.json 2> $O/bench_prev.err
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_new2.json 2> $O/bench_new2.err
P="timeout -s KILL 90 rocprofv3 --output-format csv"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $O/p1 -o run -- python3 tools/lagw_bench.py > $O/p1.log 2>&1
echo done
