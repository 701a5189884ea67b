# Round-6: the whole GPU suite on one box (one pytest process), then smoke().
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-suite}; mkdir -p $O
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/suite.log 2>&1
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo done
