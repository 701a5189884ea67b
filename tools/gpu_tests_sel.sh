# Selected GPU tests: bash tools/gpu_tests_sel.sh OUTDIR 'pytest args...'
set -e
export TMPDIR=/tmp
O=gpurun_out/$1; shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread --durations=15 -p no:cacheprovider "$@" > $O/tests.log 2>&1
