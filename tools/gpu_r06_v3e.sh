# Round-6: structured Gram with the next K-step's fragments read ahead of the MFMAs
# (SGLM_LAGW_PF=1, default) against reads at their MFMAs (=0): parity tests, standalone timing,
# SQ wait/issue counters, in-process interleaved C4 grid A/B.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-v3e}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_laggram_w.py > $O/tests.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_pf.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 SGLM_LAGW_PF=0 python3 tools/lagw_bench.py > $O/time_nopf.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/sq1 -o run -- python3 tools/lagw_bench.py > $O/sq1.log 2>&1
timeout -k 10 600 python3 tools/grid_ab.py 6 pf:env.SGLM_LAGW_PF=1 nopf:env.SGLM_LAGW_PF=0 > $O/ab_pf.json 2> $O/ab_pf.err
echo done
