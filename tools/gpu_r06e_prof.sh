# Round-6b artifacts (after the first-iteration dedup, the column windows and the deferred inversion): the structured Gram's HBM traffic in the C4 grid (separate FETCH / WRITE
# passes) and its instruction mix (SQ passes), the default bench line (CPU baseline at three
# lambdas, drop-in flow), the product-only kernel-trace summary, the mixed / production-flow /
# logged-workload lines and the simulated rank shares.  Output under gpurun_out/${1:-p6e}.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-p6e}; mkdir -p $O
B="python3 bench.py --steps 1 --warmup 0 --no-cpu --no-dropin --no-check"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $B > $O/write.log 2>&1
python3 tools/pmc_traffic.py $O/fetch $O/write $O/r06e_pmc_traffic.json --kernel lag_gram_w2_kernel > $O/pmc.log 2>&1
cp $O/r06e_pmc_traffic.json profiles/r06e_pmc_traffic.json     # the bench line below reads it
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $O/sq1 -o run -- $B > $O/sq1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $O/sq2 -o run -- $B > $O/sq2.log 2>&1
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-check > $O/bench_prof.json 2> $O/kt.err
timeout -k 10 300 python3 bench.py --config c4mixed --no-cpu > $O/bench_c4mixed.json 2> $O/bench_c4mixed.err
timeout -k 10 400 python3 bench.py --config cbprod > $O/bench_cbprod.json 2> $O/bench_cbprod.err
timeout -k 10 300 python3 bench.py --config olsref --no-cpu > $O/bench_olsref.json 2> $O/bench_olsref.err
timeout -k 10 300 python3 bench.py --config prod50 --no-cpu > $O/bench_prod50.json 2> $O/bench_prod50.err
for w in 2 4 8; do timeout -k 10 300 python3 tools/rank_sim.py --world $w --all > $O/rank_$w.json 2> $O/rank_$w.err; done
echo done
