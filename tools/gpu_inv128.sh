# 128-tile inversion levels: the chain test, chain timings per workgroup threshold, kernel stats.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-inv128}; mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 150 --timeout-method thread -p no:cacheprovider tests/test_gpu_kernels.py -k "many_fits or chol" > $O/k.log 2>&1
for t in 0 256 512 1024; do
  SGLM_INV128_WG=$t timeout -k 10 200 python -u tools/chol_bench.py --n 1 6 11 20 --reps 10 > $O/chain_$t.json 2> $O/chain_$t.err
done
SGLM_INV128_WG=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt0 -o run -- python3 tools/chol_bench.py --n 20 --reps 5 > $O/kt0.json 2> $O/kt0.err
SGLM_INV128_WG=256 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt256 -o run -- python3 tools/chol_bench.py --n 20 --reps 5 > $O/kt256.json 2> $O/kt256.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu > $O/c4_bench.json 2> $O/c4.err
