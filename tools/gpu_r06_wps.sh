# Round-6: the structured Gram at one wave per SIMD (4 x 4 tiles per wave, fragment prefetch)
# against two waves per SIMD: correctness, standalone timing, C4 grid.  Output gpurun_out/$1.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-wps}; mkdir -p $O
timeout -k 10 300 env SGLM_LAGW_WPS1=1 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_laggram_w.py > $O/tests_wps1.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_wps2.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LAGW_WPS1=1 python3 tools/lagw_bench.py > $O/time_wps1.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_wps2.json 2> $O/bench_wps2.err
timeout -k 10 300 env SGLM_LAGW_WPS1=1 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench_wps1.json 2> $O/bench_wps1.err
P="timeout -s KILL 90 rocprofv3 --output-format csv"
export SGLM_LAGW_WPS1=1     # inherited by the profiled program (nothing but python3 after --)
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $O/p1 -o run -- python3 tools/lagw_bench.py > $O/p1.log 2>&1
echo done
