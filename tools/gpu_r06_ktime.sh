# Round-6: the bench's kernel-only Gram timing against the rocprofv3 kernel summary of the same
# command.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-ktime}; mkdir -p $O
timeout -k 10 300 python3 bench.py --no-cpu --no-dropin --no-check > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-dropin --no-check > $O/bench_prof.json 2> $O/kt.err
echo done
