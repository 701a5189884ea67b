# Round-3 check: the whole GPU suite (full-size 20-lambda parity, real 2-rank process group),
# smoke, the default bench line and a 2-rank gloo rehearsal of the sharded bench.  A test
# assertion failure (pytest rc 1) still lets the bench run; any other failure (crash, GPU
# fault, timeout) ends the script.
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r03a}
mkdir -p $O
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=30 -p no:cacheprovider > $O/tests.log 2>&1 || rc=$?
echo "pytest rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --no-cpu > $O/bench_g2_gloo.json 2> $O/bench_g2_gloo.err
exit $rc
