# Round-6: IRLS fit groups (one host thread + stream per group, their chains overlapping the
# other group's main-stream work) and concurrent chains against the default, in one process.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-grp}; mkdir -p $O
timeout -k 10 500 python3 -u tools/grid_ab.py 6 base: g2:IRLS_GROUPS=2 g2s:IRLS_GROUPS=2,GROUP_SPLIT=snake g3s:IRLS_GROUPS=3,GROUP_SPLIT=snake cs2:CHOL_SPLIT=2 > $O/ab.json 2> $O/ab.err
echo done
