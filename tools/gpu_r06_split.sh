# Round-6: structured Gram with split heavy pieces (second halves added by the symmetrize
# pass): parity tests, standalone timing split / no split, per-workgroup timeline, in-process
# interleaved C4 grid A/B.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-split}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_laggram_w.py tests/test_gpu_mixed_structured.py > $O/tests.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_split.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LAGW_SPLIT=0 python3 tools/lagw_bench.py > $O/time_nosplit.log 2>&1
timeout -k 10 200 env LAGW_REPS=2 SGLM_LIB=$V/libsglm_trace.so SGLM_LAGW_TRACE_OUT=$O/tr python3 tools/lagw_bench.py > $O/time_trace.log 2>&1
python3 tools/lagw_trace.py $O/tr > $O/summary_trace.json
rm -f $O/tr_*.bin
timeout -k 10 600 python3 tools/grid_ab.py 6 split:env.SGLM_LAGW_SPLIT=1 nosplit:env.SGLM_LAGW_SPLIT=0 > $O/ab_split.json 2> $O/ab_split.err
echo done
