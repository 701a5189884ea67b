# Round-6b: the first iteration's 20-fit chain as two concurrent chains (CHOL_SPLIT=2 for
# batches of >= 12 new factorisations), a longer interleaved A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-split3}; mkdir -p $O
timeout -k 10 700 python3 -u tools/grid_ab.py 14 base: cs2m12:CHOL_SPLIT=2,CHOL_SPLIT_MIN=12 > $O/ab.json 2> $O/ab.err
echo done
