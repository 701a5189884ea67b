# Round-6: per-workgroup timelines of the structured Gram probe builds: full kernel, no staging
# in the loop (p1), no MFMA (p2) -- timing only, results invalid in p1 / p2.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-trace2}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
for v in trace trace_p1 trace_p2; do
timeout -k 10 200 env LAGW_REPS=2 SGLM_LIB=$V/libsglm_$v.so SGLM_LAGW_TRACE_OUT=$O/$v python3 tools/lagw_bench.py > $O/time_$v.log 2>&1
python3 tools/lagw_trace.py $O/$v > $O/summary_$v.json
rm -f $O/${v}_*.bin
done
echo done
