set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-lagpmc}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d $O/p1 -o run -- python3 tools/lag_bench.py 120 lag > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU --output-format csv -d $O/p2 -o run -- python3 tools/lag_bench.py 120 lag > $O/p2.log 2>&1
