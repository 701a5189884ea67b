# Round-6 diagnostics of the structured Gram (sglm_lag_gram_w) on the C4 design: timing with the
# development probes (1 = no H stores, 2 = no global loads, 3 = both), then separate PMC passes
# (instruction mix, LDS, vector-memory path, L2, HBM fetch / write).  Output gpurun_out/${1:-lw}.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-lw}; mkdir -p $O
timeout -k 10 200 env LAGW_PROBES=0,1,2,3 python3 tools/lagw_bench.py > $O/time.log 2>&1
P="timeout -s KILL 90 rocprofv3 --output-format csv"
B="python3 tools/lagw_bench.py"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU -d $O/p1 -o run -- $B > $O/p1.log 2>&1
$P --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR -d $O/p2 -o run -- $B > $O/p2.log 2>&1
$P --pmc TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_TOTAL_CACHE_ACCESSES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ TCP_READ_TAGCONFLICT_STALL_CYCLES -d $O/p3 -o run -- $B > $O/p3.log 2>&1
$P --pmc TCC_HIT TCC_MISS -d $O/p4 -o run -- $B > $O/p4.log 2>&1
$P --pmc FETCH_SIZE -d $O/p5 -o run -- $B > $O/p5.log 2>&1
$P --pmc WRITE_SIZE -d $O/p6 -o run -- $B > $O/p6.log 2>&1
echo done
