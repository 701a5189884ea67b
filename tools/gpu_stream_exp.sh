# Where the factorisation chain runs (SGLM_CHOL_STREAM side / prio / serial): C4 bench line and
# the slowest simulated 8-rank share per mode.   Usage: bash tools/gpu_stream_exp.sh
set -e
export TMPDIR=/tmp
O=gpurun_out/sexp; mkdir -p $O
for m in side prio serial; do
  SGLM_CHOL_STREAM=$m timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu > $O/bench_$m.json 2> $O/bench_$m.err
  SGLM_CHOL_STREAM=$m timeout -k 10 300 python -u tools/rank_sim.py --world 8 --rank 2 > $O/rank8_$m.json 2> $O/rank8_$m.err
done
