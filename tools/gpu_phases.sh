set -e
export TMPDIR=/tmp
O=gpurun_out/ph; mkdir -p $O
timeout -k 10 300 python tools/grid_phases.py > $O/phases.json 2> $O/phases.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err
timeout -k 10 300 python tools/rank_sim.py --world 8 --all > $O/all8.log 2>&1
