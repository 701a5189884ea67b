# Round-6: inverse columns with direct launches (no chain graph) vs the graph
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-invcol2}; mkdir -p $O
SGLM_CHOL_GRAPH=0 timeout -k 10 300 python3 -u tools/chol_bench.py --n 1 3 20 --env SGLM_INV_COL=1,0 > $O/chain_nograph.json 2> $O/chain_nograph.err
timeout -k 10 300 python3 -u tools/chol_bench.py --n 1 3 20 --env SGLM_INV_COL=1,0 > $O/chain_graph.json 2> $O/chain_graph.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 tools/chol_bench.py --n 1 --reps 5 --env SGLM_INV_COL=1 > $O/kt.log 2>&1
echo done
