# Round-6 structured Gram v2 (one staging register set): tests, timing v2 vs v1, kernel trace,
# PMC, and the C4 bench line.  Output gpurun_out/${1:-lw4}.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-lw4}; mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_laggram_w.py > $O/tests.log 2>&1
timeout -k 10 200 env LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_v2.log 2>&1
timeout -k 10 200 env SGLM_LAGW_V1=1 LAGW_REPS=6 python3 tools/lagw_bench.py > $O/time_v1.log 2>&1
P="timeout -s KILL 90 rocprofv3 --output-format csv"
B="python3 tools/lagw_bench.py"
$P --kernel-trace --stats -d $O/kt -o run -- $B > $O/kt.log 2>&1
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $O/p1 -o run -- $B > $O/p1.log 2>&1
$P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR -d $O/p2 -o run -- $B > $O/p2.log 2>&1
$P --pmc FETCH_SIZE -d $O/p5 -o run -- $B > $O/p5.log 2>&1
$P --pmc WRITE_SIZE -d $O/p6 -o run -- $B > $O/p6.log 2>&1
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin > $O/bench.json 2> $O/bench.err
timeout -k 10 300 env SGLM_LAGW_V1=1 python3 bench.py --no-cpu --no-dropin > $O/bench_v1.json 2> $O/bench_v1.err
echo done
