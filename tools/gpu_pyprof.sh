# Host-side Python profile of the C4 bench (one IRLS group, so the host path is serial).
set -e
export TMPDIR=/tmp
O=gpurun_out/pyprof; mkdir -p $O
SGLM_IRLS_GROUPS=1 timeout -k 10 300 python -u -m cProfile -o $O/bench.prof bench.py --steps 3 --warmup 1 --no-cpu > $O/bench.json 2> $O/bench.err
python -c "
import pstats
p = pstats.Stats('$O/bench.prof')
p.sort_stats('tottime').print_stats(40)
" > $O/tottime.txt
python -c "
import pstats
p = pstats.Stats('$O/bench.prof')
p.sort_stats('cumulative').print_stats(60)
" > $O/cumtime.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/kt.json 2> $O/kt.err
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_plain.json 2> $O/bench_plain.err
