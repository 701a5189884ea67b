# Round-6b: the factorisation chain's side stream at high priority, and look-ahead depths, at the
# deduped grid (one process, alternating grids)
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-prio}; mkdir -p $O
timeout -k 10 700 python3 -u tools/grid_ab.py 8 base: prio:CHOL_STREAM=prio la2:env.SGLM_CHOL_LOOKAHEAD=2 la6:env.SGLM_CHOL_LOOKAHEAD=6 prio_la6:CHOL_STREAM=prio,env.SGLM_CHOL_LOOKAHEAD=6 > $O/ab.json 2> $O/ab.err
echo done
