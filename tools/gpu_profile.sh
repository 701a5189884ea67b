# Round artifacts: PMC traffic of the Gram (separate FETCH/WRITE passes), the default bench line
# (with CPU baseline), the rocprofv3 kernel-trace summary of the same bench command, the C5,
# session-prep, signal and design-matrix bench lines, a 2-rank gloo rehearsal of the sharded
# bench on the one GPU (fit and row sharding), and simulated 2/4/8-rank shares of both modes.  Everything lands under
# gpurun_out/prof (merged back by gpurun); copy what is judged into profiles/ afterwards.
# Usage on the box: bash tools/gpu_profile.sh ROUND   (e.g. r02)
set -e
export TMPDIR=/tmp
R=${1:-r02}
O=gpurun_out/prof; mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu > $O/write.log 2>&1
python tools/pmc_traffic.py $O/fetch $O/write $O/${R}_pmc_traffic.json > $O/pmc.log 2>&1
cp $O/${R}_pmc_traffic.json profiles/${R}_pmc_traffic.json     # the bench line below reads it
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/kt.err
timeout -k 10 300 python bench.py --config c5 > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 python bench.py --config prep > $O/bench_prep.json 2> $O/bench_prep.err
timeout -k 10 300 python bench.py --config signal > $O/bench_signal.json 2> $O/bench_signal.err
timeout -k 10 300 python bench.py --config designmat > $O/bench_designmat.json 2> $O/bench_designmat.err
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --no-cpu > $O/bench_g2_gloo.json 2> $O/bench_g2_gloo.err
for w in 2 4 8; do
  timeout -k 10 300 python -u tools/rank_sim.py --world $w --all > $O/rank$w.json 2> $O/rank$w.err
  timeout -k 10 300 python -u tools/rank_sim.py --mode rows --world $w --all > $O/rows$w.json 2> $O/rows$w.err
done
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --shard rows --no-cpu > $O/bench_g2_gloo_rows.json 2> $O/bench_g2_gloo_rows.err
