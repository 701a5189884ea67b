set -e
export TMPDIR=/tmp
O=gpurun_out/chk; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python tools/rank_sim.py --world 8 --all > $O/all8.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/rank_sim.py --world 8 --rank 2 > $O/r2.log 2>&1
