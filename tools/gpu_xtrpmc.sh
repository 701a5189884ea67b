# PMC passes over the gradient micro-benchmark (four-panel kernel at 120 fits).
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-xtrpmc}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/p1 -o run -- python3 tools/lag_bench.py 120 bits > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/p2 -o run -- python3 tools/lag_bench.py 120 bits > $O/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/p3 -o run -- python3 tools/lag_bench.py 120 bits > $O/p3.log 2>&1
