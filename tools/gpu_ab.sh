# A/B of engine knobs on one box: chain timings and C4 bench lines, alternating the variants.
# Usage: bash tools/gpu_ab.sh
set -e
export TMPDIR=/tmp
O=gpurun_out/ab; mkdir -p $O
timeout -k 10 120 python -u tools/chol_bench.py > $O/chain_base.json 2> $O/chain_base.err
SGLM_INV_LDS=1 timeout -k 10 120 python -u tools/chol_bench.py > $O/chain_lds.json 2> $O/chain_lds.err
SGLM_INV_LDS=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread -k chol > $O/tests_lds.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_base_$rep.json 2> $O/bench_base_$rep.err
  SGLM_DIAG4=0 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_d1_$rep.json 2> $O/bench_d1_$rep.err
  SGLM_INV_LDS=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_lds_$rep.json 2> $O/bench_lds_$rep.err
done
