# Round-6: per-workgroup timeline of the structured Gram (probe build) on the C4 design.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-trace}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
timeout -k 10 200 env LAGW_REPS=3 SGLM_LIB=$V/libsglm_trace.so SGLM_LAGW_TRACE_OUT=$O/tr python3 tools/lagw_bench.py > $O/time.log 2>&1
python3 tools/lagw_trace.py $O/tr > $O/summary.json
rm -f $O/tr_*.bin
echo done
