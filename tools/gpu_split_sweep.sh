# Gram v6 minimum split-K sweep on the C4 bench (grid wall per setting).
set -e
export TMPDIR=/tmp
O=gpurun_out/split; mkdir -p $O
for s in 1 2 4; do
  SGLM_SYRK6_MIN_SPLIT=$s timeout -k 10 240 python bench.py --steps 3 --warmup 1 --no-cpu > $O/b$s.json 2> $O/b$s.err
done
