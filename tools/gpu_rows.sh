# Row-sharded grid check: the sharding tests (real 2/3-rank gloo groups on the one GPU, replay
# determinism), the simulated 2/4/8-rank row-slab shares and a 2-rank gloo bench rehearsal.
set -e
export TMPDIR=/tmp
O=gpurun_out/rows; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
for w in 2 4 8; do
  timeout -k 10 300 python -u tools/rank_sim.py --mode rows --world $w --all > $O/rows$w.json 2> $O/rows$w.err
done
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --no-cpu --steps 5 > $O/g2.json 2> $O/g2.err
