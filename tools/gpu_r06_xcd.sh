# Round-6: structured Gram with every piece of an event on one XCD (SGLM_LAGW_XCD=1, default)
# against the plain job order (=0): HBM traffic (FETCH / WRITE passes of the standalone launches),
# timing, timeline, parity tests, in-process interleaved C4 grid A/B.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-xcd}; mkdir -p $O
V=sabatinilab-glm_amd/sglm_hip/variants
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_laggram_w.py > $O/tests.log 2>&1
for x in 1 0; do
export SGLM_LAGW_XCD=$x
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch$x -o run -- python3 tools/lagw_bench.py > $O/fetch$x.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write$x -o run -- python3 tools/lagw_bench.py > $O/write$x.log 2>&1
python3 tools/pmc_traffic.py $O/fetch$x $O/write$x $O/traffic$x.json --kernel lag_gram_w2_kernel > $O/traffic$x.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time$x.log 2>&1
timeout -k 10 200 env LAGW_REPS=2 SGLM_LIB=$V/libsglm_trace.so SGLM_LAGW_TRACE_OUT=$O/tr$x python3 tools/lagw_bench.py > $O/time_trace$x.log 2>&1
python3 tools/lagw_trace.py $O/tr$x > $O/summary_trace$x.json
rm -f $O/tr${x}_*.bin
done
unset SGLM_LAGW_XCD
timeout -k 10 600 python3 tools/grid_ab.py 6 xcd:env.SGLM_LAGW_XCD=1 plain:env.SGLM_LAGW_XCD=0 > $O/ab_xcd.json 2> $O/ab_xcd.err
echo done
