# Round check: parity tests, smoke, then the profile artifacts (PMC traffic, bench line, kernel-trace stats).
set -e
export TMPDIR=/tmp
O=gpurun_out/full
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/gpu_profile.sh ${1:-r03}
