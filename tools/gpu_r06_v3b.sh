# Round-6: structured Gram v3 staging without splits -- parity tests, standalone timing against
# the previous library, SQ instruction mix of the standalone launches, C4 grids interleaved.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-v3b}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_laggram_w.py > $O/tests.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_new.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LIB=$V/libsglm_prev.so python3 tools/lagw_bench.py > $O/time_prev.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/sq1 -o run -- python3 tools/lagw_bench.py > $O/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq2 -o run -- python3 tools/lagw_bench.py > $O/sq2.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_new.json 2> $O/bench_new.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_prev.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_prev.json 2> $O/bench_prev.err
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_new2.json 2> $O/bench_new2.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_prev.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_prev2.json 2> $O/bench_prev2.err
echo done
