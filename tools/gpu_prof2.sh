set -e
export TMPDIR=/tmp
O=gpurun_out/prof2; mkdir -p $O
timeout -k 10 300 python tools/grid_phases.py > $O/phases.json 2> $O/phases.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/p1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p8 -o run -- python3 tools/rank_sim.py --world 8 --rank 2 > $O/r2.json 2> $O/p8.err
