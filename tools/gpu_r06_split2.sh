# Round-6b: concurrent factorisation chains (CHOL_SPLIT) at the deduped grid, where the first
# iteration's 20-fit chain runs beside an almost idle main stream
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-split2}; mkdir -p $O
timeout -k 10 600 python3 -u tools/grid_ab.py 8 base: cs2:CHOL_SPLIT=2 cs3:CHOL_SPLIT=3 cs2m10:CHOL_SPLIT=2,CHOL_SPLIT_MIN=12 > $O/ab.json 2> $O/ab.err
echo done
