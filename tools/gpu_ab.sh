# A/B of engine knobs on one box: chain timings, parity tests under the variant, and C4 bench
# lines alternating the variants.   Usage: bash tools/gpu_ab.sh VAR=VALUE
set -e
export TMPDIR=/tmp
KV=${1:-SGLM_UPD_LDS=1}
O=gpurun_out/ab_${KV//[=.]/_}; mkdir -p $O
timeout -k 10 120 python -u tools/chol_bench.py > $O/chain_base.json 2> $O/chain_base.err
env $KV timeout -k 10 120 python -u tools/chol_bench.py > $O/chain_var.json 2> $O/chain_var.err
env $KV timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_var.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_base_$rep.json 2> $O/bench_base_$rep.err
  env $KV timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_var_$rep.json 2> $O/bench_var_$rep.err
done
env $KV timeout -k 10 300 python -u tools/rank_sim.py --world 8 --all > $O/rank8_var.json 2> $O/rank8_var.err
