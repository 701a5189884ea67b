# Simulated rank shares at head: row-sharded (replay) and fit-sharded, 2/4/8 ranks
set -e
export TMPDIR=/tmp
O=gpurun_out/rows2; mkdir -p $O
for w in 2 4 8; do
  timeout -k 10 300 python -u tools/rank_sim.py --mode rows --world $w --all > $O/rows$w.json 2> $O/rows$w.err
  timeout -k 10 300 python -u tools/rank_sim.py --world $w --all > $O/fits$w.json 2> $O/fits$w.err
done
