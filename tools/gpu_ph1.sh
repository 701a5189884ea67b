set -e
export TMPDIR=/tmp
O=gpurun_out/ph1; mkdir -p $O
SGLM_IRLS_GROUPS=1 timeout -k 10 300 python tools/grid_phases.py > $O/phases.json 2> $O/phases.err
SGLM_IRLS_GROUPS=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/b.json 2> $O/b.err
