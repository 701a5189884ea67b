# Chain as a cached HIP graph vs direct launches (SGLM_CHOL_GRAPH is read once per process):
# alternating processes on one box
set -e
export TMPDIR=/tmp
O=gpurun_out/gab; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python -u tools/grid_ab.py 3 graph: > $O/graph_$rep.json 2> $O/graph_$rep.err
  SGLM_CHOL_GRAPH=0 timeout -k 10 200 python -u tools/grid_ab.py 3 direct: > $O/direct_$rep.json 2> $O/direct_$rep.err
done
