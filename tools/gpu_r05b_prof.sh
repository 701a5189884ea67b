# Round-5 artifacts after the event-structured Gram (sglm_lag_gram_w): its HBM traffic (separate
# FETCH / WRITE passes), the default bench line, the product-only kernel-trace summary, and the
# OLS / production-grid / mixed bench lines.  Output under gpurun_out/p5b.
set -e
export TMPDIR=/tmp
O=gpurun_out/p5b; mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-dropin --no-check > $O/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-dropin --no-check > $O/write.log 2>&1
python tools/pmc_traffic.py $O/fetch $O/write $O/r05b_pmc_traffic.json --kernel lag_gram_w_kernel > $O/pmc.log 2>&1
cp $O/r05b_pmc_traffic.json profiles/r05b_pmc_traffic.json     # the bench line below reads it
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-check > $O/bench_prof.json 2> $O/kt.err
timeout -k 10 300 python bench.py --config olsref --no-cpu > $O/bench_olsref.json 2> $O/bench_olsref.err
timeout -k 10 300 python bench.py --config prod50 --no-cpu > $O/bench_prod50.json 2> $O/bench_prod50.err
timeout -k 10 300 python bench.py --config c4mixed --no-cpu > $O/bench_c4mixed.json 2> $O/bench_c4mixed.err
