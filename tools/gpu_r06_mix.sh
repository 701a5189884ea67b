# Round-6: K-unroll variants of the structured Gram (standalone + C4 grid), then the new parity
# tests (mixed structured path, cb production flow, LagFrame as a DataFrame) and the drop-in
# profile.  Output gpurun_out/${1:-mx}.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-mx}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_u2.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LIB=$V/libsglm_u4.so python3 tools/lagw_bench.py > $O/time_u4.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LIB=$V/libsglm_u8.so python3 tools/lagw_bench.py > $O/time_u8.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_u2.json 2> $O/bench_u2.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_u4.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_u4.json 2> $O/bench_u4.err
timeout -k 10 300 env SGLM_LIB=$V/libsglm_u8.so python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_u8.json 2> $O/bench_u8.err
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_lagframe.py tests/test_gpu_cbflow.py tests/test_gpu_mixed_structured.py > $O/tests.log 2>&1 || echo "tests failed" >> $O/tests.log
timeout -k 10 300 python3 tools/dropin_prof.py c4 > $O/dropin_prof.log 2>&1
echo done
