# Round-4 artifacts: gradient PMC (new default vs the round-3 one-group kernel), the Gram's HBM
# traffic (separate FETCH / WRITE passes), simulated 2/4/8-rank shares, the full bench line.
set -e
export TMPDIR=/tmp
O=gpurun_out/p4; mkdir -p $O
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/xtr_new -o run -- python3 tools/lag_bench.py 120 bits > $O/xtr_new.log 2>&1
SGLM_XTR_PIPE=0 SGLM_XTR_NGW=1 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/xtr_r03 -o run -- python3 tools/lag_bench.py 120 bits > $O/xtr_r03.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-dropin > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-dropin > $O/write.log 2>&1
python tools/pmc_traffic.py $O/fetch $O/write $O/r04_pmc_traffic.json > $O/pmc.log 2>&1
for w in 2 4 8; do
  timeout -k 10 300 python -u tools/rank_sim.py --world $w --all > $O/rank$w.json 2> $O/rank$w.err
done
timeout -k 10 500 python bench.py > $O/bench_full.json 2> $O/bench_full.err
