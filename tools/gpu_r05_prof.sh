# Round-5 artifacts: the Gram's HBM traffic (separate FETCH / WRITE passes), the default bench
# line (C4 + drop-in + full-fold CPU baseline), the kernel-trace summary of the product alone
# (--no-check: the f64 Newton-distance check kernels stay out), the design-matrix, OLS and mixed
# bench lines.  Everything lands under gpurun_out/p5; copy what is judged into profiles/.
set -e
export TMPDIR=/tmp
O=gpurun_out/p5; mkdir -p $O
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-dropin --no-check > $O/fetch.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-dropin --no-check > $O/write.log 2>&1
python tools/pmc_traffic.py $O/fetch $O/write $O/r05_pmc_traffic.json > $O/pmc.log 2>&1
cp $O/r05_pmc_traffic.json profiles/r05_pmc_traffic.json     # the bench line below reads it
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-check > $O/bench_prof.json 2> $O/kt.err
timeout -k 10 300 python bench.py --config designmat > $O/bench_designmat.json 2> $O/bench_designmat.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dm -o run -- python3 bench.py --config designmat --steps 3 --warmup 1 --no-cpu > $O/bench_designmat_prof.json 2> $O/dm.err
timeout -k 10 300 python bench.py --config c4mixed --no-cpu > $O/bench_c4mixed.json 2> $O/bench_c4mixed.err
