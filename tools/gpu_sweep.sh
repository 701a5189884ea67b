set -e
export TMPDIR=/tmp
O=gpurun_out/sweep; mkdir -p $O
timeout -k 10 500 python tools/syrk_sweep.py > $O/sweep.log 2>&1
