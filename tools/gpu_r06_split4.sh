# Round-6b: chain-split variants around the default (CHOL_SPLIT=2 for >= 12 new factors)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-split4}; mkdir -p $O
timeout -k 10 800 python3 -u tools/grid_ab.py 10 base: m8:CHOL_SPLIT_MIN=8 s3:CHOL_SPLIT=3 s3m18:CHOL_SPLIT=3,CHOL_SPLIT_MIN=18 > $O/ab.json 2> $O/ab.err
echo done
